"""Write tests/golden/oracle_golden.npz from the CPU oracle (test infrastructure).

    python tools/make_golden.py

The fixtures pin the oracle across rounds (tests/test_oracle.py) and are the
committed expected outputs the GPU parity test checks the HIP path against
(tests/test_gpu_parity.py::test_gpu_against_committed_golden).  The oracle
itself is pinned by the reference's known-answer tests and by the independent
Python restatement (tests/pyref.py) -- see DESIGN.md, "Oracle".
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from tools_golden import CASES, GOLDEN_PATH, run_case  # noqa: E402


def main():
    out = {}
    for name in CASES:
        for k, v in run_case(name).items():
            out[f"{name}/{k}"] = v
        print(name, {k: v.shape for k, v in run_case(name).items()})
    np.savez_compressed(GOLDEN_PATH, **out)
    print("wrote", GOLDEN_PATH, os.path.getsize(GOLDEN_PATH), "bytes")


if __name__ == "__main__":
    main()
