#!/bin/bash
# Round 4, one box: the full GPU suite (in-tree: D0), then the cfg4 walker A/B (D0: effects
# deferred to k_final, per-thread walkers only; DL32 / DL96: + the pipelined long-component walker
# for components of 32 / 96 events or more, on a second stream), then cfg4's trace.
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4/pytest_full.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|error" gpurun_out/r4/pytest_full.log | head -20; tail -5 gpurun_out/r4/pytest_full.log; exit 1; }
tail -2 gpurun_out/r4/pytest_full.log
VARIANTS="D0 DL32 DL96" bash tools/ab.sh cfg4 2 > gpurun_out/r4/ab_cfg4_walker_defer2.txt 2>&1 || { echo "walker ab failed"; tail -5 gpurun_out/r4/ab_cfg4_walker_defer2.txt; exit 1; }
cat gpurun_out/r4/ab_cfg4_walker_defer2.txt
cp tigerbeetle_amd/libtbgpu.so /tmp/keep.so && cp tigerbeetle_amd/libtbgpu_DL32.so tigerbeetle_amd/libtbgpu.so && bash tools/gpu_r4_trace_cfg4.sh; cp /tmp/keep.so tigerbeetle_amd/libtbgpu.so
