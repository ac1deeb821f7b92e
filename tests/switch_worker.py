"""Child process of test_small_n_switch_off_paths: runs the small-N step
sequences (tests/small_n_steps.py) on the oracle and on the product library
under the environment it was started with, and prints one JSON line
{sequence: [indices of differing objects]}.  Test infrastructure only."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from hectr_amd.gpqhe import Engine  # noqa: E402
from tests.small_n_steps import SEQUENCES, mismatches  # noqa: E402


def main():
    ora, prod = Engine.oracle(), Engine.product()
    out = {name: mismatches(f(ora), f(prod)) for name, f in SEQUENCES.items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
