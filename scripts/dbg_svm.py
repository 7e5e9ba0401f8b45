"""Debug: MFMA vs VALU SVM kernel vs oracle on a 3-class OvO model with missing values."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from flink_jpmml_amd.bench.synth import stream_matrix, svm_pmml
from flink_jpmml_amd.runtime.compiled import CompiledPmml

c = CompiledPmml.from_string(svm_pmml(n_features=12, n_sv=160, seed=6, n_classes=3, gamma=0.2))
plan = c.plan(torch.device("cuda:0"))
X = stream_matrix(30_000, 12, seed=3, missing_rate=0.01)
s, v = plan.score(X)
s, v = s.cpu().numpy(), v.cpu().numpy().astype(bool)
ref, vref = c.score_matrix_oracle(X)
bad = np.nonzero(v != vref)[0]
print("mfma: mismatched valid", len(bad), "kernel valid", v.sum(), "oracle valid", vref.sum())
nanrow = np.isnan(X).any(axis=1)
print("rows with NaN", nanrow.sum(), "mismatch rows with NaN", nanrow[bad].sum())
print("first bad rows", bad[:10], "v", v[bad[:10]], "vref", vref[bad[:10]], "rowmod256", bad[:10] % 256)
plan.n_svp = 0
s2, v2 = plan.score(X)
s2, v2 = s2.cpu().numpy(), v2.cpu().numpy().astype(bool)
print("valu: mismatched valid", (v2 != vref).sum(), "score agree", (s2[v2] == ref[v2]).mean())
print("mfma vs valu score agree", (s[v & v2] == s2[v & v2]).mean())
