#!/bin/bash
# One GPU lease, parameterised: runs the named steps in order, each under its own time limit, and
# stops at the first failure (set -e).  Output goes to gpurun_out/<TAG>_*.
#
#   bash tools/gpu_lease.sh TAG STEP [STEP ...]
#
# steps:
#   tests[:K]        pytest -m gpu (only tests matching -k K when given)
#   smoke            __graft_entry__.smoke()
#   bench            the default bench line (stdout json + detail)
#   prof             rocprofv3 --kernel-trace --stats of the bench, then the FETCH_SIZE / WRITE_SIZE /
#                    FP64 passes (one counter group per run) -> make_traffic.py input
#   kstats:LEG       rocprofv3 --kernel-trace --stats of one leg (summary via tools/kstats.py)
#   pmc:LEG          the counter groups below over one leg (join | table | ranges | hist | sort | z3 | xz | query)
#   ab:LEG:LIBS      alternating runs of one leg over variant libraries (geomesa_amd/lib/<lib>.so,
#                    comma-separated; "prod" = the product library), 3 rounds
#   probe:NAME       python tools/NAME.py $PROBE_ARGS (ranges_probe, hist_probe, sort_probe, query_probe, ...)
#   abprobe:NAME:LIBS  the probe over variant libraries (as ab), 3 rounds, into one text file
#   kprobe:NAME:LIB  rocprofv3 --kernel-trace --stats of one probe run with one library (prod = shipped)
set -e
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
out=gpurun_out/$tag

leg_args() {   # the bench arguments of one leg
  case $1 in
    join) echo "--only join --no-cpu --no-gather --steps 1 --warmup 0 --join-steps 3" ;;
    ranges) echo "--only extra --no-cpu --no-gather --steps 2 --warmup 1" ;;
    table) echo "--only z3,table --no-cpu --steps 2 --warmup 1" ;;   # the table's keys come from the z3 leg
    z3) echo "--only z3 --no-cpu --steps 10 --warmup 2" ;;
    extra) echo "--only extra --no-cpu --steps 6 --warmup 1" ;;
    *) echo "--no-cpu" ;;
  esac
}

for step in "$@"; do
  name=${step%%:*}; arg=${step#*:}; [ "$arg" = "$step" ] && arg=""
  echo "[$(date +%T)] $step" >> ${out}_steps.log
  case $name in
    tests)
      if [ -n "$arg" ]; then kk=(-k "$arg"); else kk=(); fi
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v "${kk[@]}" --timeout 300 --timeout-method thread \
        > ${out}_tests.log 2>&1 ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > ${out}_smoke.log 2>&1 ;;
    n2)   # the N > 1 paths with two ranks on the box's one GPU and gloo collectives (reduced sizes)
      GM_BENCH_DEVICE=0 GM_BENCH_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 \
        --join-steps 2 --points 250000000 --join-points 250000000 --table-rows 100000000 \
        > ${out}_n2.json 2> ${out}_n2.err
      cp gpurun_out/bench_detail_n2.json ${out}_n2_detail.json ;;
    bench)
      timeout -k 10 600 python -u bench.py > ${out}_bench.json 2> ${out}_bench.err
      cp gpurun_out/bench_detail_n1.json ${out}_bench_detail.json ;;
    prof)
      timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d ${out}_prof -o run -- \
        python3 bench.py --steps 10 --join-steps 3 --no-cpu > ${out}_prof_bench.json 2> ${out}_prof.err
      i=0
      rq="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
      for g in FETCH_SIZE WRITE_SIZE "$rq"; do
        timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv --pmc $g -d ${out}_pmc/p$i -o run -- \
          python3 bench.py --only z3,extra,table --no-cpu --steps 2 --warmup 1 > ${out}_pmc$i.log 2>&1
        i=$((i+1))
      done
      for g in FETCH_SIZE WRITE_SIZE SQ_INSTS_VALU_FLOPS_FP64 "$rq"; do
        timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv --pmc $g -d ${out}_pmc/p$i -o run -- \
          python3 bench.py --only join --no-cpu --steps 1 --warmup 0 --join-steps 1 > ${out}_pmc$i.log 2>&1
        i=$((i+1))
      done ;;
    tpmc)   # the traffic-calibration probe: its own timing, then one counter group per rocprofv3 pass
      timeout -k 10 120 tools/traffic_probe > ${out}_tprobe.txt 2>&1
      i=0
      for g in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" FETCH_SIZE WRITE_SIZE \
               "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_HIT_sum TCC_MISS_sum"; do
        timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc $g -d ${out}_tpmc/p$i -o run -- \
          tools/traffic_probe > ${out}_tpmc_p$i.log 2>&1
        i=$((i+1))
      done ;;
    kstats)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d ${out}_kstats_$arg -o run -- \
        python3 bench.py $(leg_args $arg) > ${out}_kstats_$arg.json 2> ${out}_kstats_$arg.err
      python3 tools/kstats.py ${out}_kstats_$arg > ${out}_kstats_$arg.txt 2>&1 || true ;;
    pmc)
      groups=(
        "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
        "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS"
        "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_VMEM"
        "TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TD_TC_STALL_sum"
        "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum"
        "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"
        "FETCH_SIZE"
        "WRITE_SIZE"
      )
      if [ -n "$PMC_GROUPS" ]; then IFS=";" read -ra groups <<< "$PMC_GROUPS"; fi
      cmd="python3 bench.py $(leg_args $arg)"
      [ "$arg" = ranges ] && cmd="python3 tools/ranges_probe.py 100000"
      [ "$arg" = hist ] && cmd="python3 tools/hist_probe.py"
      [ "$arg" = sort ] && cmd="python3 tools/sort_probe.py"
      [ "$arg" = xz ] && cmd="python3 tools/xz_probe.py"
      [ "$arg" = query ] && cmd="python3 tools/query_probe.py"
      mkdir -p ${out}_pmc_$arg
      i=0
      for g in "${groups[@]}"; do
        timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv --pmc $g -d ${out}_pmc_$arg/p$i -o run -- \
          $cmd > ${out}_pmc_$arg/p$i.log 2>&1 || { echo "pass $i ($g) failed: $?" >> ${out}_pmc_$arg/failed.txt; exit 1; }
        i=$((i+1))
      done ;;
    vpmc)   # counter groups (PMC_GROUPS, ';'-separated, or the read-request sizes + hits / misses) over one leg,
            # once per variant library: vpmc:LEG:lib1,lib2,...
      leg=${arg%%:*}; libs=${arg#*:}
      if [ -n "$PMC_GROUPS" ]; then IFS=";" read -ra vgroups <<< "$PMC_GROUPS"
      else vgroups=("TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
                    "TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"); fi
      for lib in ${libs//,/ }; do
        if [ "$lib" = prod ]; then unset GEOMESA_HIP_LIB; else export GEOMESA_HIP_LIB=$PWD/geomesa_amd/lib/$lib.so; fi
        i=0
        for g in "${vgroups[@]}"; do
          timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv --pmc $g -d ${out}_vpmc_${lib}/p$i -o run -- \
            python3 bench.py $(leg_args $leg) > ${out}_vpmc_${lib}_p$i.log 2>&1
          i=$((i+1))
        done
      done
      unset GEOMESA_HIP_LIB ;;
    ab)
      leg=${arg%%:*}; libs=${arg#*:}
      aout=${out}_$leg   # one record set per leg (several ab steps in one lease)
      for r in 1 2 3; do
        for lib in ${libs//,/ }; do
          if [ "$lib" = prod ]; then unset GEOMESA_HIP_LIB; else export GEOMESA_HIP_LIB=$PWD/geomesa_amd/lib/$lib.so; fi
          timeout -k 10 300 python -u bench.py $(leg_args $leg) > ${aout}_ab_${lib}_$r.json 2> ${aout}_ab_${lib}_$r.err
          cp gpurun_out/bench_detail_n1.json ${aout}_ab_${lib}_$r.detail.json
        done
      done
      unset GEOMESA_HIP_LIB
      python3 tools/show_ab.py ${aout}_ab > ${aout}_ab.txt ;;
    probe)
      timeout -k 10 400 python -u tools/$arg.py $PROBE_ARGS > ${out}_$arg.txt 2>&1 ;;
    abprobe)
      pname=${arg%%:*}; libs=${arg#*:}
      for r in 1 2 3; do
        for lib in ${libs//,/ }; do
          if [ "$lib" = prod ]; then unset GEOMESA_HIP_LIB; else export GEOMESA_HIP_LIB=$PWD/geomesa_amd/lib/$lib.so; fi
          echo "== $lib round $r" >> ${out}_abprobe_$pname.txt
          timeout -k 10 300 python -u tools/$pname.py $PROBE_ARGS >> ${out}_abprobe_$pname.txt 2>&1
        done
      done
      unset GEOMESA_HIP_LIB ;;
    kprobe)
      pname=${arg%%:*}; lib=${arg#*:}
      if [ "$lib" = prod ]; then unset GEOMESA_HIP_LIB; else export GEOMESA_HIP_LIB=$PWD/geomesa_amd/lib/$lib.so; fi
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d ${out}_kprobe_${pname}_$lib -o run -- \
        python3 tools/$pname.py $PROBE_ARGS > ${out}_kprobe_${pname}_$lib.txt 2>&1
      unset GEOMESA_HIP_LIB
      python3 tools/kstats.py ${out}_kprobe_${pname}_$lib >> ${out}_kprobe_${pname}_$lib.txt 2>&1 || true ;;
    *)
      echo "unknown step $step" >&2; exit 2 ;;
  esac
done
