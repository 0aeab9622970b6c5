#!/bin/bash
# A/B: run the headline bench against alternative library builds in exp/<variant>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in "$@"; do
  v=${spec%%:*}; extra=""; [ "$spec" != "$v" ] && extra="--nodes ${spec#*:}"
  if [ "$v" = "main" ]; then dir=""; else dir="$PWD/exp/$v"; fi
  SHIRLEY_LIB_DIR=$dir timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu $extra > gpurun_out/ab_$v.log 2>&1
  rc=$?
  echo "$spec rc=$rc $(tail -1 gpurun_out/ab_$v.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], "Msamples/s", d["roofline"]["kernel_ms"], "ms")' 2>/dev/null)"
  [ $rc -eq 0 ] || exit $rc
done
