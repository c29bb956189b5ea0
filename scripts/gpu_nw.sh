#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 600 python -m pytest tests -m gpu -q -x > /tmp/pytest_gpu.log 2>&1
rc=$?; tail -2 /tmp/pytest_gpu.log; [ $rc -eq 0 ] || { grep -v "^Extension" /tmp/pytest_gpu.log | tail -30; exit $rc; }
for nw in 4 8 16; do
  RS_FM_NW=$nw timeout -k 10 120 python scripts/diag_launch.py 2>&1 | grep embed_fm | sed "s/^/nw=$nw /" || exit 3
done
echo DONE
