# Full GPU test suite (one process), then smoke(), on one box
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/r5tests
timeout -k 10 960 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5tests/pytest.log 2>&1 || { tail -40 gpurun_out/r5tests/pytest.log; exit 3; }
tail -3 gpurun_out/r5tests/pytest.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5tests/smoke.log 2>&1 || { tail -20 gpurun_out/r5tests/smoke.log; exit 4; }
cat gpurun_out/r5tests/smoke.log
