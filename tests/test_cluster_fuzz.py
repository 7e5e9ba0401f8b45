"""Randomized ClusteringModels on the device vs the float64 oracle: every distance metric, a random
compareFunction per field (absDiff, gaussSim with a similarityScale, delta, equal — ties in the
inputs make delta / equal bite), field weights, missing values (the PMML missing-value weight
adjustment) and 1-200 clusters, on the automatic plan (VALU kernel or the exact-fp32 MFMA kernel).
The predicted cluster must match the oracle on every row with a clear winner (the fp64 runner-up
trails by more than fp32 resolution); validity exactly."""

import re

import numpy as np
import pytest

from tests._suite import gpu_seeds

from flink_jpmml_amd.runtime.compiled import CompiledPmml

METRICS = ["squaredEuclidean", "euclidean", "cityBlock", "chebychev", 'minkowski p-parameter="3"']
COMPARES = ["absDiff", "gaussSim", "delta", "equal"]


def _case(seed: int):
    from flink_jpmml_amd.bench.synth import kmeans_pmml

    rng = np.random.default_rng(4400 + seed)
    F = int(rng.choice([1, 3, 8, 20]))
    K = int(rng.choice([1, 5, 40, 200]))
    metric = METRICS[seed % len(METRICS)]
    txt = kmeans_pmml(n_clusters=K, n_features=F, seed=seed, metric=metric, weighted=bool(rng.integers(2)))
    mixed = rng.random() < 0.6
    if mixed:  # a random compareFunction per field
        def sub(m):
            cf = str(rng.choice(COMPARES))
            extra = f' similarityScale="{rng.uniform(0.5, 2.0):.3f}"' if cf == "gaussSim" else ""
            return f'<ClusteringField field="{m.group(1)}" compareFunction="{cf}"{extra}'
        txt = re.sub(r'<ClusteringField field="(f\d+)" compareFunction="absDiff"', sub, txt)
    return txt, F, mixed


def _inputs(n: int, F: int, seed: int) -> np.ndarray:
    from flink_jpmml_amd.bench.synth import stream_matrix

    rng = np.random.default_rng(seed)
    X = stream_matrix(n, F, seed=seed, missing_rate=0.05)
    r = rng.random(X.shape) < 0.3
    X[r] = np.round(X[r])  # ties with the rounded centres are rare; exact 0 / ±1 values are not
    return X


@pytest.mark.parametrize("seed", range(10))
def test_random_clusterings_lower(seed):
    from flink_jpmml_amd.runtime.plans import lowering_dry_run

    txt, _, _ = _case(seed)
    with lowering_dry_run():
        CompiledPmml.from_string(txt).plan("cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("seed", gpu_seeds(30, 10))
def test_random_clusterings_on_gpu(gpu, seed):
    txt, F, mixed = _case(seed)
    c = CompiledPmml.from_string(txt)
    plan = c.plan(gpu)
    X = _inputs(6000, F, seed)
    s, v = plan.score(X)
    s, v = s.cpu().numpy().astype(np.float64), v.cpu().numpy().astype(bool)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all(), (seed, type(plan).__name__)
    if not v.any():
        return
    # rows whose fp64 winner leads by less than fp32 resolution are ties for an fp32 kernel (e.g. a
    # gaussSim component far below the delta components' sum): compare the clear rows only
    ev = c.evaluator
    P, _ = c.prepare(X)
    D = np.sort(ev.distances(ev.feature_matrix(c.columns(P))), axis=1)
    if not ev.kind_distance:
        D = -D[:, ::-1]
    gap = (D[:, 1] - D[:, 0]) / np.maximum(1e-30, np.abs(D[:, 0])) if D.shape[1] > 1 else np.ones(len(X))
    clear = v & (gap > 1e-5)  # chebychev over delta / equal fields: mostly ties
    if clear.any():
        assert (s[clear] == ref[clear]).mean() >= 0.999, (seed, type(plan).__name__, mixed)
