#!/bin/bash
# r06 session zh: the whole GPU suite and smoke() on the round's last tree.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so oracle/*.so
export TMPDIR=/tmp
O=gpurun_out/r06zh
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > $O/suite.log 2>&1
rc=$?; tail -3 $O/suite.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
