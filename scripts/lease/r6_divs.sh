#!/bin/bash
# Round 6: igemm_conv_kernel with float-reciprocal pixel splits -- numerics
# suites, then the default dgrad / fp4-forward times of every E18 shape.
set -u
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/gpu/test_bconv_bwd_kernels.py tests/gpu/test_fp4_forward.py tests/gpu/test_conv_family.py tests/gpu/test_pointwise.py tests/gpu/test_conv3x3.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_divs.log 2>&1 || exit 1
for op in dgrad fwd4; do
  timeout -k 10 300 python3 tools/one_conv.py --op $op --shape all --batch 1536 --reps 10 2>&1 | grep us/call >> gpurun_out/divs.log || exit 1
done
