# Round 6: grid cap of the bf16 BN backward dx kernels (temporary knob
# ZK_BN_DX_GRID in norm_pool.hip rows_grid; default 2048), tools/bn_lab.py, same box.
set -o pipefail
for gcap in 2048 512 1024 4096 2048; do
  ZK_BN_DX_GRID=$gcap timeout -k 10 200 python -u tools/bn_lab.py --tag d$gcap --json gpurun_out/bn_lab_dx.jsonl > gpurun_out/bn_lab_d$gcap.log 2>&1 || exit $?
done
