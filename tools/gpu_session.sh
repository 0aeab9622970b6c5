#!/bin/bash
# One gpurun session: smoke -> GPU parity tests -> short bench.  Every GPU step has its own time
# limit; after a crash / timeout nothing more touches the GPU (test *failures* do not stop it).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  return $rc
}
rocm-smi --showproductname > gpurun_out/device.txt 2>&1
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
run gpu_tests 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
run bench_spp50 300 python bench.py --spp 50 --steps 2 --warmup 1 --no-cpu || exit 1
run bench_full 600 python bench.py --steps 2 --warmup 1 || exit 1
