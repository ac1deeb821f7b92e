"""Config 2 alone (NTT -> INTT roundtrip of 1024 polys at N=2^16, L=8, the
bench's < 2^51 primes) for a rocprofv3 kernel trace / PMC pass:
    rocprofv3 --kernel-trace --stats -d ... -- python scripts/prof_ntt.py
"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from bench import ntt_roundtrip  # noqa: E402
from hectr_amd.gpqhe import Engine  # noqa: E402

polys = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
eng = Engine.product()
eng.init_params(logn=16, nlimbs=8, dnum=2, nspecial=4, slots=64, q0_bits=51, qi_bits=50, p_bits=51, seed=1)
stream = torch.cuda.Stream()
eng.lib.gpqhe_set_stream(ctypes.c_void_p(stream.cuda_stream))
print(json.dumps(ntt_roundtrip(eng, stream, 16, 8, polys, reps=2)))
eng.exit()
