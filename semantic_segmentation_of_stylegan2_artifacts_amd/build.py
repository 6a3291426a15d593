"""Build the gfx950 HIP library ``libmsunet_hip.so`` in-tree (no JIT cache, no torch types).

    python -m semantic_segmentation_of_stylegan2_artifacts_amd.build [--force]

Each ``csrc/*.hip`` is compiled separately with ``hipcc --offload-arch=gfx950`` (in
parallel) and linked into one shared library next to this file, so it travels to the GPU
box with the repo snapshot.
"""
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "_build")
LIB = os.path.join(HERE, "libmsunet_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# -amdgpu-mfma-vgpr-form: MFMA accumulators in VGPRs.  In the default AGPR form the register
# allocator shuffled accumulators between AGPRs and VGPRs inside the main loops (68 v_accvgpr
# moves per 42 MFMAs in the weight-gradient loop, 300-500 per NT / token GEMM kernel); gfx950
# MFMAs read and write either file at the same rate.  Same-box r04f: weight gradient -9 %,
# bench 169.1 / 169.1 / 169.5 vs 168.1 / 167.8 / 167.9 img/s.
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
         "-munsafe-fp-atomics", "-mllvm", "-amdgpu-mfma-vgpr-form=1"]


def _sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def _headers():
    return sorted(glob.glob(os.path.join(CSRC, "*.h")))


def _stale(obj, src):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(f) > t for f in [src] + _headers())


def _compile(src):
    obj = os.path.join(BUILD, os.path.basename(src).replace(".hip", ".o"))
    cmd = [HIPCC] + FLAGS + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
    return obj


def build(force=False, jobs=None):
    os.makedirs(BUILD, exist_ok=True)
    srcs = _sources()
    objs = [os.path.join(BUILD, os.path.basename(s).replace(".hip", ".o")) for s in srcs]
    todo = [s for s, o in zip(srcs, objs) if force or _stale(o, s)]
    if todo:
        jobs = jobs or min(len(todo), max(1, min(8, os.cpu_count() or 1)))
        with cf.ThreadPoolExecutor(jobs) as ex:
            list(ex.map(_compile, todo))
    if todo or not os.path.exists(LIB) or any(os.path.getmtime(o) > os.path.getmtime(LIB) for o in objs):
        tmp = LIB + ".tmp"
        cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", tmp] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
        os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
