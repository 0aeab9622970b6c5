#!/bin/bash
# A/B of bench flag sets on the current build: each argument is one quoted flag set.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
for flags in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu $flags > gpurun_out/abf_$i.log 2>&1
  rc=$?
  echo "[$flags] rc=$rc $(tail -1 gpurun_out/abf_$i.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], "Msamples/s", d["roofline"]["kernel_ms"], "ms", c.get("rounds"), c.get("kernel_ms_split"))' 2>/dev/null)"
  [ $rc -eq 0 ] || { tail -3 gpurun_out/abf_$i.log; exit $rc; }
done
