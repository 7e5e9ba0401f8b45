"""Dump device vs oracle chain results for one fuzz seed (diagnostics for tests/test_chain_fuzz.py)."""
import sys

import numpy as np
import torch

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
from test_chain_fuzz import _doc, _inputs  # noqa: E402

from flink_jpmml_amd.runtime.compiled import CompiledPmml  # noqa: E402

for seed in (19, 37):
    c = CompiledPmml.from_string(_doc(seed))
    plan = c.plan(torch.device("cuda:0"))
    X = _inputs(8000, seed)
    s, v = plan.score(X)
    np.savez(f"gpurun_out/chain_diag/seed{seed}.npz", X=X, s=s.cpu().numpy(), v=v.cpu().numpy())
    print(seed, "saved")
