#!/bin/bash
# Round-2 session M (final state of the round): -m gpu suite + smoke, the default bench line, rocprofv3
# kernel stats + HBM PMC of the headline (profiles/r02).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests \
  > gpurun_out/m_tests.log 2>&1
rc=$?; tail -n 3 gpurun_out/m_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/m_smoke.log 2>&1 || exit $?
tail -n 1 gpurun_out/m_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/m_bench.log 2>&1 || exit $?
tail -n 1 gpurun_out/m_bench.log | cut -c1-300
bash tools/profile.sh r02m --steps 3 --warmup 1 --no-cpu --no-configs
