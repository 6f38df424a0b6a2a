"""Builds libgeomesa_hip.so in-tree for gfx950 (hipcc, -ffp-contract=off: the JVM never fuses)."""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = ["gm_ctx.hip", "gm_curve.hip", "gm_filter.hip", "gm_pip_build.hip", "gm_pip_join.hip", "gm_pip_relate.hip", "gm_pip_query.hip", "gm_ranges.hip", "gm_sort.hip", "gm_arrow.hip", "gm_stats.hip", "gm_legacy.hip"]
OUT = os.path.join(HERE, "lib", "libgeomesa_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-fPIC",
         "-Wall", "-Wno-unused-function"]


VARIANT_ONLY = ("GM_JX_", "GM_NO_REF_CHECKS")


def sources():
    return [os.path.join(HERE, "csrc", s) for s in SRC if os.path.exists(os.path.join(HERE, "csrc", s))]


def needs_build():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = sources() + [os.path.join(HERE, "csrc", f) for f in os.listdir(os.path.join(HERE, "csrc"))]
    deps.append(os.path.join(os.path.dirname(HERE), "include", "geomesa_hip.h"))
    return any(os.path.getmtime(f) > t for f in deps)


def build(force=False, verbose=True, out=OUT, defines=()):
    """Compile every HIP unit into one shared library; `defines` builds a tuning variant (e.g.
    GM_JILP=8) to another path for side-by-side measurement."""
    if out == OUT and not defines and not force and not needs_build():
        return OUT
    if out == OUT and any(d.startswith(VARIANT_ONLY) for d in defines):
        # timing variants (stage ablations, checks compiled out, measured-and-dropped layouts): never
        # in the shipped library
        raise ValueError("timing-variant defines %s cannot be built into %s; pass --out=<other path>"
                         % ([d for d in defines if d.startswith(VARIANT_ONLY)], OUT))
    if out == OUT:
        defines = tuple(defines) + ("GM_PRODUCT_BUILD",)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    # one object per unit, compiled in parallel (no device code crosses units), then one link
    objdir = out + ".objs"
    os.makedirs(objdir, exist_ok=True)
    defs = ["-D" + d for d in defines]

    def compile_one(src):
        obj = os.path.join(objdir, os.path.basename(src) + ".o")
        cmd = [HIPCC] + FLAGS + defs + ["-c", "-o", obj, src]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd)
        return obj

    jobs = max(1, min(len(sources()), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4))))
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(compile_one, sources()))
    cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out + ".tmp"] + objs
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    args = sys.argv[1:]
    defs = [a[2:] for a in args if a.startswith("-D")]
    outs = [a.split("=", 1)[1] for a in args if a.startswith("--out=")]
    build(force="--force" in args, out=outs[0] if outs else OUT, defines=defs)
