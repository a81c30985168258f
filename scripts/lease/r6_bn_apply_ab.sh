# Round 6: ResNet-50 b1024 with the bf16 BN apply's grid cap at 2048 (old) vs
# 65536 (ZK_BN_APPLY_GRID, temporary knob), alternating on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
for cap in 2048 65536 2048 65536; do
  ZK_BN_APPLY_GRID=$cap timeout -k 10 400 python -u bench.py --model ResNet50 --batch 1024 --steps 20 > gpurun_out/r50_cap$cap.log 2>&1 || exit $?
  echo "cap $cap $(tail -1 gpurun_out/r50_cap$cap.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
