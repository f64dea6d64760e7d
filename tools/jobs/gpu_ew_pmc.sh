# HBM-bound kernels: timing (tools/bench_ew.py) and the bytes the L2 actually fetched / wrote
# (TCC FETCH_SIZE / WRITE_SIZE, one pass each) -> achieved bandwidth per kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/ewpmc
timeout -k 10 200 python -u tools/bench_ew.py > gpurun_out/ewpmc/time.json 2>&1 || { tail -5 gpurun_out/ewpmc/time.json; exit 2; }
tail -1 gpurun_out/ewpmc/time.json
i=0
for P in "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d gpurun_out/ewpmc/p$i -o p -- python3 tools/bench_ew.py > gpurun_out/ewpmc/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 gpurun_out/ewpmc/p$i.log; exit 3; }
done
python tools/pmc_db_summary.py $(find gpurun_out/ewpmc -name "*.db") --filter "" > gpurun_out/ewpmc/summary.txt 2>&1
grep -A4 "swiglu\|norm_\|adamw\|colsum" gpurun_out/ewpmc/summary.txt | head -80
find gpurun_out/ewpmc -name "*.db" -delete
