"""Randomized shapes of the other model families on the GPU with the automatic plan choice vs the
float64 oracle: SVMs (four kernels, binary / one-against-one up to 12 classes / regression, 4 to
1100 support vectors), k-means (five metrics, field weights, 1 to 300 clusters), k-NN
(classification / regression, k 1-7) and segmented MiningModels (every aggregation method, 2 to
90 segments, with and without segment predicates). Each case: validity equal to the oracle,
scores within fp32 of it (labels: near-boundary rows may flip). The plan must lower
(``NotLowerable`` fails the case instead of a silent host fallback)."""

import numpy as np
import pytest

from tests._suite import gpu_seeds

pytestmark = pytest.mark.gpu


def _check(c, plan, X, label: bool, rtol=1e-4, agree=0.99):
    s, v = plan.score(X)
    s, v = s.cpu().numpy().astype(np.float64), v.cpu().numpy().astype(bool)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all()
    if not v.any():
        return
    if label:
        assert (s[v] == ref[v]).mean() >= agree
    else:
        scale = max(1.0, float(np.abs(ref[v]).max()))
        np.testing.assert_allclose(s[v], ref[v], rtol=0, atol=rtol * scale)


@pytest.mark.parametrize("seed", gpu_seeds(24, 8))
def test_random_svms(gpu, seed):
    from flink_jpmml_amd.bench.synth import stream_matrix, svm_pmml
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    rng = np.random.default_rng(8000 + seed)
    kernel = ["linear", "polynomial", "radialBasis", "sigmoid"][seed % 4]
    classes = int(rng.choice([0, 2, 3, 5, 12]))
    F = int(rng.choice([2, 16, 64, 130]))
    n_sv = int(rng.choice([4, 40, 300, 1100]))
    gamma = float(rng.choice([0.5, 0.05, 0.005])) / max(1.0, F / 16)
    txt = svm_pmml(n_features=F, n_sv=n_sv, seed=seed, kernel=kernel, classification=classes > 0, gamma=gamma,
                   n_classes=max(classes, 2))
    c = CompiledPmml.from_string(txt)
    plan = c.plan(gpu)
    X = stream_matrix(int(rng.choice([1, 300, 6000])), F, seed=seed, missing_rate=0.01)
    _check(c, plan, X, label=classes > 0, rtol=2e-4, agree=0.98)


@pytest.mark.parametrize("seed", gpu_seeds(20, 6))
def test_random_kmeans(gpu, seed):
    from flink_jpmml_amd.bench.synth import kmeans_pmml, stream_matrix
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    rng = np.random.default_rng(8100 + seed)
    metric = ["squaredEuclidean", "euclidean", "cityBlock", "chebychev", 'minkowski p-parameter="3"'][seed % 5]
    K = int(rng.choice([1, 7, 64, 300]))
    F = int(rng.choice([1, 4, 32, 100]))
    c = CompiledPmml.from_string(kmeans_pmml(n_clusters=K, n_features=F, seed=seed, metric=metric,
                                             weighted=bool(rng.integers(2))))
    plan = c.plan(gpu)
    X = stream_matrix(int(rng.choice([1, 500, 8000])), F, seed=seed, missing_rate=0.0)
    _check(c, plan, X, label=True, agree=0.995)


@pytest.mark.parametrize("seed", gpu_seeds(16, 6))
def test_random_knn(gpu, seed):
    from flink_jpmml_amd.bench.synth import knn_pmml, stream_matrix
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    rng = np.random.default_rng(8200 + seed)
    cls = bool(seed % 2)
    k = int(rng.choice([1, 3, 7]))
    F = int(rng.choice([2, 8, 20]))
    txt = knn_pmml(n_instances=int(rng.choice([10, 200, 1000])), n_features=F, k=k, classification=cls, seed=seed,
                   metric=["euclidean", "squaredEuclidean", "cityBlock"][seed % 3])
    c = CompiledPmml.from_string(txt)
    plan = c.plan(gpu)
    X = stream_matrix(int(rng.choice([1, 400, 5000])), F, seed=seed, missing_rate=0.0)
    _check(c, plan, X, label=cls, rtol=1e-4, agree=0.99)


_REG = ["selectFirst", "max", "min", "median", "sum", "average", "weightedAverage"]
_CLS = ["majorityVote", "weightedMajorityVote", "selectFirst", "average", "weightedAverage", "max", "median"]


@pytest.mark.parametrize("seed", gpu_seeds(24, 8))
def test_random_segmentations(gpu, seed):
    from flink_jpmml_amd.bench.synth import segmented_pmml, stream_matrix
    from flink_jpmml_amd.runtime.compiled import CompiledPmml

    rng = np.random.default_rng(8300 + seed)
    cls = bool(seed % 2)
    method = (_CLS if cls else _REG)[int(rng.integers(7))]
    F = int(rng.choice([3, 6, 20]))
    txt = segmented_pmml(method=method, classification=cls, n_segments=int(rng.choice([2, 8, 40, 90])),
                         depth=int(rng.integers(2, 6)), n_features=F, n_classes=int(rng.choice([2, 3, 12])),
                         seed=seed, predicates=bool(rng.integers(2)))
    c = CompiledPmml.from_string(txt)
    plan = c.plan(gpu)
    X = stream_matrix(int(rng.choice([1, 700, 9000])), F, seed=seed, missing_rate=0.05)
    _check(c, plan, X, label=cls, rtol=1e-4, agree=0.99)
