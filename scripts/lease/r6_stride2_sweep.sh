#!/bin/bash
# Round 6: standalone sweep of the stride-2 transition convs' data-gradient and
# fp4-forward tile variants at batch 1536 (tools/one_conv.py), one line per run
# into gpurun_out/s2.log.
set -u
export TMPDIR=/tmp
out=gpurun_out/s2.log
for v in -1 4 5 6 7 8 9 42 43 48; do
  timeout -k 10 120 python3 tools/one_conv.py --op dgrad --shape 56,56,64,128,2 --batch 1536 --variant $v --reps 10 2>&1 | grep -E "us/call|Error" >> $out || true
done
for v in -1 0 1 2 3 10 11 16 40 41 44 46; do
  timeout -k 10 120 python3 tools/one_conv.py --op dgrad --shape 28,28,128,256,2 --batch 1536 --variant $v --reps 10 2>&1 | grep -E "us/call|Error" >> $out || true
done
for v in -1 0 1 4 6 7 8 9; do
  timeout -k 10 120 python3 tools/one_conv.py --op fwd4 --shape 56,56,64,128,2 --batch 1536 --variant $v --reps 10 2>&1 | grep -E "us/call|Error" >> $out || true
done
