"""bench.py's secondary_c1_solo alone: the reference's AAPL d/w/m 8-kernel sweep, one GPR at a time
(GPR/model_trainer.py:14-20), GPU vs the CPU oracle. usage: python tools/c1_sweep.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

if __name__ == "__main__":
    print(json.dumps(bench.secondary_c1_solo(0)), flush=True)
