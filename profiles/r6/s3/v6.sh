#!/bin/bash
# r6 session 3, V6: issue cost of the fp32 march's VALU mix at 1 and 2 waves/SIMD
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r6v6
mkdir -p $O
timeout -k 10 60 ./tools/pk_issue_probe > $O/pk_issue.txt 2>&1
rc=$?; cat $O/pk_issue.txt; exit $rc
