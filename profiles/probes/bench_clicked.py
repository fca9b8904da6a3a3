"""Probe: bench.py with another history length (measurement only, not the
headline workload). NRMS_PROBE_CLICKED=n sets the clicked titles per
impression; the rest of the command line is bench.py's.

    NRMS_PROBE_CLICKED=32 python profiles/probes/bench_clicked.py --no-cpu-baseline --no-extras
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

bench.N_CLICKED = int(os.environ.get("NRMS_PROBE_CLICKED", bench.N_CLICKED))
if __name__ == "__main__":
    bench.main()
