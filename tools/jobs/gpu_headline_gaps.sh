# GPU idle gaps in the headline step (rocprofv3 kernel trace of bench.py, 3 timed steps)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/hgaps; mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace -d $O/trace -o run -- python3 bench.py --steps 3 --warmup 2 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 3; }
DB=$(find $O/trace -name "*.db" | head -n 1)
python3 tools/gaps.py "$DB" --top 30 --min_us 100 > $O/gaps.txt
rm -rf $O/trace
cat $O/gaps.txt | head -60
