#!/bin/bash
# Interleaved bench A/B on one box: every argument is one configuration
# (comma-separated bench.py arguments, '-' for the defaults); the whole list
# runs ROUNDS times (default 2) so drift shows up.  One JSON line per run in
# gpurun_out/ab.jsonl, tagged with its configuration.
#   gpurun -- bash scripts/ab.sh - --data,pool --rt,wgrad_reduce=slab
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out
mkdir -p "$OUT"
STEPS=${AB_STEPS:-100}
ROUNDS=${AB_ROUNDS:-2}
for r in $(seq 1 "$ROUNDS"); do
  i=0
  for cfg in "$@"; do
    i=$((i + 1))
    args=""
    [ "$cfg" != "-" ] && args="${cfg//,/ }"
    log="$OUT/ab_r${r}_c${i}.log"
    echo "start r$r c$i [$cfg] $(date +%T)" >> "$OUT/progress.txt"
    timeout -k 10 300 python -u bench.py --steps "$STEPS" --warmup 10 $args \
      --json-out "$OUT/ab_tmp.json" > "$log" 2>&1
    rc=$?
    echo "done r$r c$i rc=$rc $(date +%T)" >> "$OUT/progress.txt"
    if [ $rc -ne 0 ]; then exit $rc; fi
    python -c "import json,sys; d=json.load(open('$OUT/ab_tmp.json')); d['ab']={'round':$r,'cfg':'$cfg'}; print(json.dumps(d))" >> "$OUT/ab.jsonl"
  done
done
