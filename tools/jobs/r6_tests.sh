# Round 6: full GPU suite (one process) + smoke()
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/r6final
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r6final/pytest.log 2>&1 || { tail -40 gpurun_out/r6final/pytest.log; exit 3; }
tail -1 gpurun_out/r6final/pytest.log
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6final/smoke.log 2>&1 || { tail -20 gpurun_out/r6final/smoke.log; exit 4; }
grep -c "smoke ok" gpurun_out/r6final/smoke.log
