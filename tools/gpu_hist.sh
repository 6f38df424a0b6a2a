cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_stats.py -x -v --timeout 120 --timeout-method thread > gpurun_out/h1_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --only z3,extra --no-cpu --steps 10 > gpurun_out/h1_bench.json 2> gpurun_out/h1_bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/h1_prof -o run -- python3 bench.py --only z3,extra --no-cpu --steps 6 > gpurun_out/h1_prof.json 2> gpurun_out/h1_prof.err
