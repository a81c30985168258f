# Round 6: bf16 BN dx grid caps (new: 1024 mask / 512 recomputed-ReLU) vs the old
# 2048 (ZK_BN_DX_GRID=2048, temporary knob): tools/bn_lab.py, then ResNet-50 and
# QuickNet-Large b1024 alternating on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/bn_lab.py --tag new --json gpurun_out/bn_lab_dxnew.jsonl > gpurun_out/bn_lab_dxnew.log 2>&1 || exit $?
run() {  # tag env-value model batch steps
  if [ "$2" = new ]; then unset ZK_BN_DX_GRID; else export ZK_BN_DX_GRID=$2; fi
  timeout -k 10 400 python -u bench.py --model $3 --batch $4 --steps $5 > gpurun_out/ab_$1.log 2>&1 || exit $?
  echo "$1 $(tail -1 gpurun_out/ab_$1.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
run r50_old1 2048 ResNet50 1024 20
run r50_new1 new ResNet50 1024 20
run r50_old2 2048 ResNet50 1024 20
run r50_new2 new ResNet50 1024 20
run qnl_old 2048 QuickNetLarge 1024 30
run qnl_new new QuickNetLarge 1024 30
