# full GPU suite + smoke
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/full; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
