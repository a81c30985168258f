# Round 6: BN apply / dx grid-size caps, tools/bn_lab.py, same box.  First
# run (since folded into the defaults): ZK_BN_GRID = 4096/2048 (old), 8192,
# 16384, 65536 for every apply / dx kernel.  This run: the new defaults, with
# the pooled apply's cap (ZK_BN_POOL_GRID) at 4096 (old) / 16384 / 65536.
set -o pipefail
for gcap in 4096 16384 65536; do
  ZK_BN_POOL_GRID=$gcap timeout -k 10 200 python -u tools/bn_lab.py --tag p$gcap --json gpurun_out/bn_lab_pool.jsonl > gpurun_out/bn_lab_p$gcap.log 2>&1 || exit $?
done
