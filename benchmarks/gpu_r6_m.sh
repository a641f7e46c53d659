#!/bin/bash
# round 6, call M: SQ counters of the one-tile K9d launch (where the potrf cycles go)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAVE_CYCLES \
  -d $GRAFT_REPO_ROOT/gpurun_out/r6m_pmc1 -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/benchmarks/k9d_one_tile.py 20 > $GRAFT_REPO_ROOT/gpurun_out/r6m.log 2>&1 || { tail -30 $GRAFT_REPO_ROOT/gpurun_out/r6m.log; exit 1; }
tail -2 $GRAFT_REPO_ROOT/gpurun_out/r6m.log
find $GRAFT_REPO_ROOT/gpurun_out/r6m_pmc1 -name "*counter_collection*" | head -3
