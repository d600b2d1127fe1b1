#!/bin/bash
# r03p: group sizing trace (contexts only, no LM: the load path ran fault-free in the jacobian tests)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
cat > /tmp/trace_groups.py <<'PY'
import sys, os
sys.path[:0] = ["tests", "sfm-mvs-pipeline_amd", "."]
os.environ["SFMX_BA_TRACE"] = "1"
import torch  # noqa
from diag import diagnostic
from sfmx import synth, ba
for args in [(10, 1000, 22, 1), (200, 6000, 29, 3), (200, 200000, 0xBA200, 3)]:
    p = synth.ba_problem(args[0], args[1], seed=args[2], cam_model=args[3])
    with diagnostic(SFMX_BA_TRACE="1"):
        ctx = ba.BAContext(ba.BAProblem(**p))
        ctx.close()
print("ok")
PY
timeout -k 10 120 python -u /tmp/trace_groups.py > gpurun_out/r03p_trace.log 2>&1
echo rc=$? >> gpurun_out/r03p_trace.log
