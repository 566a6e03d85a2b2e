#!/bin/bash
# Final validation of a tree on one GPU box: the GPU tests, smoke(), two bench lines and a
# rocprofv3 kernel-trace of a third.   usage: bash tools/gpu_final.sh [TAG]
set -o pipefail
O=gpurun_out/${1:-r5fin3}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 300 python bench.py > $O/bench2.json 2>> $O/bench.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu > $GRAFT_REPO_ROOT/$O/bench_prof.json 2> $GRAFT_REPO_ROOT/$O/prof.err || exit $?
