#!/bin/bash
# rocprofv3 evidence for the headline bench: one kernel-trace/stats pass, then one PMC pass per
# counter (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950; MI355X_MICROARCH.md §rocprofv3).
# Usage: tools/profile.sh <tag> [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-r01}; shift
args=${@:---steps 2 --warmup 1 --no-cpu --no-configs}
out=gpurun_out/prof_$tag
mkdir -p $out
set -o pipefail
echo "=== trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py $args \
  > $out/trace.log 2>&1 || { echo "trace failed rc=$?"; tail -20 $out/trace.log; exit 1; }
tail -2 $out/trace.log
for c in FETCH_SIZE WRITE_SIZE; do
  echo "=== pmc $c"
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $out/pmc_$c -o run -- python3 bench.py $args \
    > $out/pmc_$c.log 2>&1 || { echo "pmc $c failed rc=$?"; tail -20 $out/pmc_$c.log; exit 1; }
done
find $out -name "*.csv" | sort
