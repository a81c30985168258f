# Round 6: A/B of the 1x1 GEMM tile for N % 256 == 0, K <= 128: 41 (128x128)
# vs 43 (128x64), temporary knob ZK_PW_SMALLK, alternating on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
run() {  # tag variant args...
  local tag=$1 v=$2; shift 2
  ZK_PW_SMALLK=$v timeout -k 10 400 python -u bench.py "$@" > gpurun_out/pwab_$tag.log 2>&1 || exit $?
  echo "$tag $(tail -1 gpurun_out/pwab_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
run r50_41a 41 --model ResNet50 --batch 1024 --steps 20
run r50_43a 43 --model ResNet50 --batch 1024 --steps 20
run r50_41b 41 --model ResNet50 --batch 1024 --steps 20
run r50_43b 43 --model ResNet50 --batch 1024 --steps 20
run e18_41 41
run e18_43 43
