"""Localise MLP kernel mismatches: run a grid of shapes on the fused kernel (fp32 / bf16) and print,
per shape, how many rows disagree with the oracle in validity and value (JSON lines)."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from flink_jpmml_amd.bench.synth import mlp_pmml, stream_matrix
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    shapes = [(8, (32,)), (40, (32,)), (40, (96,)), (40, (96, 70)), (64, (256, 256)), (16, (64, 64, 64)),
              (40, (70,)), (2, (32,))]
    for prec in ("fp32", "bf16"):
        for F, hidden in shapes:
            c = CompiledPmml.from_string(mlp_pmml(n_features=F, hidden=hidden, n_out=1, seed=4))
            plan = c.plan("cuda:0", precision=prec)
            X = stream_matrix(3000, F, seed=2)
            X[5, min(3, F - 1)] = np.nan
            s, v = plan.score(X)
            s, v = s.cpu().numpy(), v.cpu().numpy()
            ref, vref = c.score_matrix_oracle(X)
            bad_v = np.nonzero(v != vref)[0]
            both = v & vref
            err = np.abs(s[both] - ref[both])
            print(json.dumps({"prec": prec, "F": F, "hidden": hidden, "valid_mismatch": int(len(bad_v)),
                              "first": bad_v[:8].tolist(), "gpu_v": v[bad_v[:8]].tolist(),
                              "gpu_s": [float(x) for x in s[bad_v[:8]]], "ref": [float(x) for x in ref[bad_v[:8]]],
                              "max_err": float(err.max()) if err.size else None,
                              "n_bad_err": int((err > 1e-3 * max(1.0, np.abs(ref[both]).max())).sum()),
                              "row5_valid": bool(v[5])}), flush=True)


if __name__ == "__main__":
    main()
