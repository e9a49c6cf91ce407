"""Builds libmahout_cms.so in-tree with hipcc for gfx950 (no JIT cache: the
.so travels with the repo snapshot to the GPU box)."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libmahout_cms.so")
SOURCES = ["cms_api.hip", "cms_ingest.hip", "cms_build.hip", "cms_partition.hip", "cms_query.hip", "cms_topk.hip", "cms_cosine_mfma.hip", "cms_cosine_sym.hip", "cms_cosine_mls.hip", "cms_profiles.hip", "cms_merge.hip", "cms_table.hip", "cms_f64.hip", "cms_output.cpp", "cms_recommend.cpp"]
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-std=c++17", "-ffp-contract=off",
         "-mcode-object-version=5", "-Wall", "-Wno-unused-function", "-I/opt/rocm/include"]


def build(verbose=False, force=False, jobs=None, defines=(), out=None):
    """CMS_BOUND_ANALYSIS=1 in the environment builds the bound-analysis
    variant (kernel parts switchable by CMS_COS_MODE; scripts/cos_modes.sh).
    Translation units compile in parallel (objects under mahout_amd/build/),
    then link into the one in-tree shared object.  `defines` + `out` build an
    A/B variant of the library elsewhere (loaded through MAHOUT_CMS_LIB)."""
    from concurrent.futures import ThreadPoolExecutor
    analysis = os.environ.get("CMS_BOUND_ANALYSIS") == "1"
    variant = bool(defines) or out is not None
    force = force or analysis or variant
    target = out or OUT
    srcs = [os.path.join(CSRC, s) for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]
    deps = srcs + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    deps.append(os.path.join(HERE, "..", "include", "mahout_cms.h"))
    if not force and os.path.exists(OUT) and all(os.path.getmtime(OUT) >= os.path.getmtime(d) for d in deps):
        return OUT
    objdir = os.path.join(HERE, "build", "variant_" + os.path.basename(target)) if variant else os.path.join(HERE, "build")
    os.makedirs(objdir, exist_ok=True)
    extra = (["-DCMS_BOUND_ANALYSIS"] if analysis else []) + ["-D" + d for d in defines]
    cflags = [f for f in FLAGS if f != "-shared"]

    def compile_one(src):
        obj = os.path.join(objdir, os.path.basename(src) + ".o")
        cmd = ["/opt/rocm/bin/hipcc"] + cflags + extra + ["-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd))
        subprocess.check_call(cmd)
        return obj

    jobs = jobs or min(len(srcs), max(1, min(16, os.cpu_count() or 1)))
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(compile_one, srcs))
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC"] + objs + [
        "-o", target, "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    return target


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--define", action="append", default=[], help="NAME=VALUE for an A/B variant")
    ap.add_argument("--out", default=None, help="variant library path")
    a = ap.parse_args()
    print(build(verbose=True, force=a.force, defines=a.define, out=a.out))
