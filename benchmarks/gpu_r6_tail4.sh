#!/bin/bash
# K9b tail (default TR = 8): tests, FID compute A/B tail on / off / on
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6_tail4
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu/test_k9b_symeig.py tests/gpu/test_k9p_pivchol.py tests/gpu/test_k9d_cholesky.py tests/metrics/image > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u benchmarks/k9b_tail_ab.py > $O/ab_on.json 2>$O/ab_on.err &&
TORCHEVAL_AMD_SYMEIG_TAIL=0 timeout -k 10 200 python -u benchmarks/k9b_tail_ab.py > $O/ab_off.json 2>$O/ab_off.err &&
timeout -k 10 200 python -u benchmarks/k9b_tail_ab.py > $O/ab_on2.json 2>$O/ab_on2.err &&
TORCHEVAL_AMD_SYMEIG_TAIL=0 timeout -k 10 200 python -u benchmarks/k9b_tail_ab.py > $O/ab_off2.json 2>$O/ab_off2.err || { cat $O/ab_*.err | tail; exit 1; }
cat $O/ab_*.json
