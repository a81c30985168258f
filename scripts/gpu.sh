#!/bin/bash
# One parameterised GPU-box driver (replaces the per-experiment one-liners).
#
#   gpurun --timeout 900 -- bash scripts/gpu.sh <step> [<step> ...]
#
# Steps (each runs under its own time limit, output under gpurun_out/):
#   tests            python -m pytest tests -m gpu
#   tests:<expr>     python -m pytest tests -m gpu -k <expr>
#   bench[:model[:batch[:steps]]]      bench.py on 1 GPU (default E18 b512 60 steps)
#   stream[:model]   bench.py --data stream (pinned ring + side-stream H2D)
#   prof[:model[:batch]]               rocprofv3 --kernel-trace --stats of bench.py
#   pmc[:model]      three rocprofv3 PMC passes over 2 training steps (SQ MFMA/LDS,
#                    FETCH_SIZE, WRITE_SIZE; one counter group per run)
#   pmcconv:op:shape[:batch] PMC passes over one conv kernel (tools/one_conv.py), e.g.
#                    pmcconv:dgrad:56,56,64,64,1:1024
#   benchargs:<a,b>  bench.py with arbitrary comma-separated arguments
#   profargs:<a,b>   rocprofv3 --kernel-trace --stats of bench.py with those arguments
#   tune[:args]      tools/tune_bconv.py with the given (comma-separated) args; '+'
#                    is a comma inside one argument (--igw,20+120)
#   py:<module>      python -m <module>  (tools, one-off diagnostics)
#   pmcpy:<script,args>  PMC passes (SQ timing, SQ instruction mix, FETCH, WRITE)
#                    over python3 <script> <args> (commas -> spaces)
#   dpgloo:<n>       bench.py with n gloo ranks sharing the GPU (ordering rehearsal)
#   env:<VAR=VAL>    export VAR=VAL for the following steps (A/B switches)
#
# A step that times out, aborts or faults ends the script (no GPU work after).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
PROG="$(pwd)/$OUT/progress.txt"

gpu_step() {
  local t=$1; shift
  local log=$1; shift
  echo "start '$*' $(date +%T)" >> "$PROG"
  timeout -k 10 "$t" "$@" > "$log" 2>&1
  local rc=$?
  echo "step '$*' rc=$rc $(date +%T)" >> "$PROG"
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -ge 128 ]; then
    echo "fatal rc=$rc in: $*" >> "$PROG"
    exit $rc
  fi
  return $rc
}

n=0
for spec in "$@"; do
  n=$((n + 1))
  IFS=':' read -r kind a1 a2 a3 <<< "$spec"
  case "$kind" in
    tests)
      if [ -n "${a1:-}" ]; then
        ZK_CURVE_DIR="$OUT/curves" gpu_step 600 "$OUT/pytest_$n.log" python -u -m pytest tests -m gpu -x -q \
          --timeout 120 --timeout-method thread -k "$a1" || exit $?
      else
        ZK_CURVE_DIR="$OUT/curves" gpu_step 900 "$OUT/pytest_$n.log" python -u -m pytest tests -m gpu -x -q \
          --timeout 120 --timeout-method thread || exit $?
      fi
      ;;
    bench)
      gpu_step 420 "$OUT/bench_${n}_${a1:-E18}.log" python -u bench.py \
        --model "${a1:-BinaryResNetE18}" --batch "${a2:-512}" --steps "${a3:-60}" \
        --warmup 10 --json-out "$OUT/bench_${n}.json" || exit $?
      ;;
    stream)
      gpu_step 420 "$OUT/stream_${n}.log" python -u bench.py --data stream \
        --model "${a1:-BinaryResNetE18}" --steps 60 --warmup 10 \
        --json-out "$OUT/stream_${n}.json" || exit $?
      ;;
    prof)
      gpu_step 600 "$OUT/prof_${n}.log" rocprofv3 --kernel-trace --stats \
        -d "$OUT/prof_$n" -o run --output-format csv -- python3 bench.py --model "${a1:-BinaryResNetE18}" \
        --batch "${a2:-512}" --steps 20 --warmup 10 --graph 0 || exit $?
      ;;
    benchargs)
      gpu_step 420 "$OUT/benchargs_${n}.log" python -u bench.py ${a1//,/ } \
        --json-out "$OUT/benchargs_${n}.json" || exit $?
      ;;
    profargs)
      gpu_step 600 "$OUT/profargs_${n}.log" rocprofv3 --kernel-trace --stats \
        -d "$OUT/profargs_$n" -o run --output-format csv -- python3 bench.py ${a1//,/ } || exit $?
      ;;
    pmc)
      R="$(pwd)"
      for pass in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS" \
                  "FETCH_SIZE" "WRITE_SIZE"; do
        tag=$(echo "$pass" | cut -d' ' -f1)
        (cd /tmp && gpu_step 150 "$R/$OUT/pmc_${n}_${tag}.log" timeout -s KILL 140 rocprofv3 --pmc $pass \
          -d "$R/$OUT/pmc_${n}_${tag}" -o run --output-format csv -- python3 "$R/bench.py" \
          --model "${a1:-BinaryResNetE18}" --steps 2 --warmup 2 --graph 0) || exit $?
      done
      ;;
    pmcconv)
      R="$(pwd)"
      nm="${a1}_${a2//,/_}"
      bt="${a3:-256}"
      nm="${nm}_b${bt}"
      gpu_step 120 "$OUT/pmcconv_${nm}_time.log" python tools/one_conv.py --op "$a1" --shape "$a2" --batch "$bt" --reps 50 || exit $?
      for pass in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT" \
                  "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
        tag=$(echo "$pass" | cut -d' ' -f1)
        (cd /tmp && gpu_step 90 "$R/$OUT/pmcconv_${nm}_${tag}.log" timeout -s KILL 80 rocprofv3 --pmc $pass \
          -d "$R/$OUT/pmcconv_${nm}_${tag}" -o run --output-format csv -- python3 "$R/tools/one_conv.py" \
          --op "$a1" --shape "$a2" --batch "$bt" --reps 5) || exit $?
      done
      ;;
    pmcpy)
      # three PMC passes over `python3 <a1 with commas as spaces>`
      R="$(pwd)"
      script="${a1%%,*}"; rest=""; [ "$script" != "$a1" ] && rest="${a1#*,}"; rest="${rest//,/ }"
      for pass in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT" \
                  "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_MFMA_MOPS_BF16" \
                  "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
        tag=$(echo "$pass" | cut -d' ' -f1)
        (cd /tmp && gpu_step 150 "$R/$OUT/pmcpy_${n}_${tag}.log" timeout -s KILL 140 rocprofv3 --pmc $pass \
          -d "$R/$OUT/pmcpy_${n}_${tag}" -o run --output-format csv -- python3 "$R/$script" $rest) || exit $?
      done
      ;;
    profpy)
      # kernel trace of python3 <a1 with commas as spaces>
      script="${a1%%,*}"; rest=""; [ "$script" != "$a1" ] && rest="${a1#*,}"; rest="${rest//,/ }"
      gpu_step 300 "$OUT/profpy_${n}.log" rocprofv3 --kernel-trace --stats \
        -d "$OUT/profpy_$n" -o run --output-format csv -- python3 "$script" $rest || exit $?
      ;;
    tune)
      targs="${a1//,/ }"  # '+' stands for a comma inside one argument (--igw 20+120)
      gpu_step 600 "$OUT/tune_${n}.log" python -u tools/tune_bconv.py ${targs//+/,} || exit $?
      ;;
    py)
      gpu_step 600 "$OUT/py_${n}.log" python -u -m "$a1" ${a2//,/ } || exit $?
      ;;
    dpgloo)
      ZK_DIST_BACKEND=gloo gpu_step 600 "$OUT/dpgloo_${n}.log" python -u bench.py \
        --gpus "${a1:-2}" --allow-shared-gpu --batch 64 --steps 10 --warmup 3 || exit $?
      ;;
    env)
      export "${spec#env:}"
      echo "env ${spec#env:}" >> "$PROG"
      ;;
    *)
      echo "unknown step $spec" >> "$PROG"; exit 2 ;;
  esac
done
echo "all steps done $(date +%T)" >> "$PROG"
