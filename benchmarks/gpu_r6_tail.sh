#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r6_tail
O=gpurun_out/r6_tail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu/test_k9b_symeig.py tests/gpu/test_k9p_pivchol.py tests/metrics/image > $O/tests.log 2>&1 &&
timeout -k 10 200 python -u benchmarks/k9b_tail_ab.py > $O/ab_on.json 2>$O/ab_on.err &&
TORCHEVAL_AMD_SYMEIG_TAIL=0 timeout -k 10 200 python -u benchmarks/k9b_tail_ab.py > $O/ab_off.json 2>$O/ab_off.err &&
timeout -k 10 200 python -u benchmarks/k9b_tail_ab.py > $O/ab_on2.json 2>$O/ab_on2.err
rc=$?
tail -3 $O/tests.log; cat $O/ab_*.json
exit $rc
