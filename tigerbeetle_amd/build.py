"""Builds libtbgpu.so in-tree for gfx950 (hipcc), and the test oracle (gcc)."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SOURCES = ["csrc/engine.hip", "csrc/workload.hip", "csrc/checksum.hip"]
HEADERS = sorted("csrc/" + f for f in os.listdir(os.path.join(HERE, "csrc")) if f.endswith((".h", ".inc"))) + [
    "../include/tb_types.h", "../include/tbg.h"]
FLAGS = ["-O3", "--offload-arch=gfx950", "-std=c++17", "-fPIC", "-shared", "-Wall"]


def build_lib(force=False):
    out = os.path.join(HERE, "libtbgpu.so")
    deps = [os.path.join(HERE, p) for p in SOURCES + HEADERS]
    if not force and os.path.exists(out) and all(os.path.getmtime(out) >= os.path.getmtime(d) for d in deps):
        return out
    tmp = out + ".tmp"  # built aside, then renamed over the library (a reader never sees a partial file)
    cmd = ["hipcc"] + FLAGS + ["-o", tmp] + [os.path.join(HERE, s) for s in SOURCES]
    subprocess.check_call(cmd, cwd=HERE)
    os.replace(tmp, out)
    return out


def build_oracle():
    subprocess.check_call(["make", "-s", "-B", "-C", os.path.join(ROOT, "oracle")])


if __name__ == "__main__":
    build_lib(force="--force" in sys.argv)
    build_oracle()
