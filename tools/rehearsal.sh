#!/bin/bash
# Multi-rank rehearsal on ONE GPU: bench.py at --gpus 4 and 8 with the gloo backend
# (ranks share the device; the exchange runs through torch.distributed, raytracer/parallel.py), both
# partitions, plus a sample partition with more ranks than samples per pixel.  Every run ends with the
# line's multi_rank_check (the multi-rank frame against one device's frame: tiles bit for bit, samples
# within 1e-12).  Output: <out>/rehearsal_<N>.jsonl, one bench line per run.
# usage: bash tools/rehearsal.sh <out dir>
out=${1:-gpurun_out/rehearsal}
mkdir -p "$out"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
run() {  # run <N> <label> <bench args...>
  local n=$1 label=$2
  shift 2
  timeout -k 10 300 python -u bench.py --gpus "$n" --dist-backend gloo --steps 2 --warmup 1 --no-cpu --no-configs "$@" \
    > "$out/rehearsal_${n}_${label}.log" 2>&1 || { echo "rehearsal $n $label failed"; tail -20 "$out/rehearsal_${n}_${label}.log"; return 1; }
  tail -1 "$out/rehearsal_${n}_${label}.log" >> "$out/rehearsal_${n}.jsonl"
  tail -1 "$out/rehearsal_${n}_${label}.log" | python3 -c 'import sys, json
d = json.loads(sys.stdin.read()); m = d["multi_rank_check"]
print(d["n_gpus"], d["config"]["ranks"], d["config"]["partition"], d["config"]["spp"], d["value"], m["status"], m["tiles"], "|", m["samples"])'
}
run 4 tiles --partition tiles &&
run 4 samples --partition samples &&
run 8 tiles --partition tiles &&
run 8 samples --partition samples &&
run 8 samples_spp4 --partition samples --spp 4
