#!/bin/bash
# BASELINE configs other than the headline, one bench run each (single GPU, megakernel).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
  tag=$1; shift
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu "$@" > gpurun_out/cfg_$tag.log 2>&1
  rc=$?
  echo "[$tag] rc=$rc $(tail -1 gpurun_out/cfg_$tag.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], "Msamples/s", d["ms_per_step"], "ms/frame", c["segments_per_sample"], "seg/sample", c["node_tests_per_segment"], "node tests/seg")' 2>/dev/null)"
  [ $rc -eq 0 ] || { tail -3 gpurun_out/cfg_$tag.log; exit $rc; }
}
run cfg1 --scene random --width 400 --aspect std16x9 --spp 50
run cfg3 --scene earth --width 800 --aspect square --spp 1000
run cfg4 --scene cornell --width 600 --aspect square --spp 10000
run cfg5_final --scene final --width 1920 --aspect std16x9 --spp 2000
run cfg5_sah --scene spheres --width 1920 --aspect std16x9 --spp 16 --bvh sah
run cfg5_ref --scene spheres --width 1920 --aspect std16x9 --spp 16 --bvh reference
