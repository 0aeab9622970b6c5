#!/bin/bash
# Round-2 session W: the default bench line, smoke, rocprofv3 kernel stats + HBM PMC and the VALU PMC
# pass of the block-segment build (profiles/r02).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/w_smoke.log 2>&1 || exit $?
tail -n 1 gpurun_out/w_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/w_bench.log 2>&1 || exit $?
tail -n 1 gpurun_out/w_bench.log | cut -c1-300
bash tools/profile.sh r02w --steps 3 --warmup 1 --no-cpu --no-configs || exit $?
bash tools/profile_valu.sh r02
