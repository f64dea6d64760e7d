"""tools/overlap.py on a synthetic rocprofv3-shaped SQLite trace (CPU)."""
import os
import sqlite3
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_overlap_tool(tmp_path):
    db = tmp_path / "t.db"
    con = sqlite3.connect(db)
    con.execute("create table kernels (kernel_name text, start integer, end integer)")
    rows = [("Cijk_gemm", 0, 1_000_000), ("Cijk_gemm", 1_500_000, 2_000_000),
            ("ncclDevKernel_Generic_AllGather_RING", 200_000, 700_000),       # fully under the GEMM
            ("ncclDevKernel_Generic_ReduceScatter_RING", 900_000, 1_600_000)]  # 0.5 ms exposed (GEMM gap)
    con.executemany("insert into kernels values (?, ?, ?)", rows)
    con.commit()
    con.close()
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "overlap.py"), str(db)],
                         capture_output=True, text=True, check=True).stdout
    assert "| rccl:allgather | 1 | 0.50 | 0.50 | 0.00 | 100.0 |" in out
    assert "| rccl:reducescatter | 1 | 0.70 | 0.20 | 0.50 | 28.6 |" in out
