"""ClusteringModel on the matrix cores (``cluster.hip::cluster_mfma_kernel``).

The MFMA path scores ``‖x‖²_w − 2 x·(w∘c) + ‖c‖²_w``; its argmin agrees with the float64 oracle's
``Σ w (x−c)²`` except on fp32 near-ties, and rows with a missing value take the exact in-kernel
fallback (so their labels match the VALU kernel's). CPU tests pin the operand packing and an fp32
numpy twin of the expansion; GPU tests compare the kernel with the oracle.
"""

import numpy as np
import pytest

from flink_jpmml_amd.bench.synth import kmeans_pmml, stream_matrix
from flink_jpmml_amd.runtime.compiled import CompiledPmml
from flink_jpmml_amd.runtime.plans import ClusterPlan


def _emulate_mfma(wc, cc, w, X, euclid):
    Xf = np.nan_to_num(X.astype(np.float32))
    xx = (w.astype(np.float32) * Xf * Xf).sum(axis=1, dtype=np.float32)
    F = X.shape[1]
    d = xx[:, None] - 2.0 * (Xf @ wc[:, :F].T) + cc[None, :]
    k = np.argmin(d, axis=1)
    best = np.maximum(d[np.arange(len(X)), k], 0.0)
    return k, (np.sqrt(best) if euclid else best)


@pytest.mark.parametrize("K,F", [(64, 32), (100, 33), (17, 7)])
def test_mfma_operands_padding(K, F):
    rng = np.random.default_rng(K)
    C, w = rng.standard_normal((K, F)), rng.uniform(0.5, 2, F)
    wc, cc = ClusterPlan.mfma_operands(C, w)
    assert wc.shape == (-(-K // 32) * 32, F + (F & 1)) and wc.dtype == np.float32
    assert np.allclose(wc[:K, :F], C * w, rtol=1e-6) and not wc[K:].any() and not wc[:, F:].any()
    assert np.allclose(cc[:K], (w * C * C).sum(1), rtol=1e-5) and np.isinf(cc[K:]).all()


@pytest.mark.parametrize("metric", ["squaredEuclidean", "euclidean"])
def test_mfma_expansion_matches_oracle(metric):
    c = CompiledPmml.from_string(kmeans_pmml(64, 32, weighted=True, metric=metric))
    ev = c.evaluator
    wc, cc = ClusterPlan.mfma_operands(ev.centers, ev.weights)
    X = stream_matrix(4000, 32, seed=3)
    ref, vref = c.score_matrix_oracle(X)
    k, _ = _emulate_mfma(wc, cc, ev.weights, X, metric == "euclidean")
    assert vref.all()
    assert (k + 1 == ref).mean() > 0.999


def _gpu_np(plan, X, **kw):
    s, v = plan.score(X, **kw)
    return s.cpu().numpy(), v.cpu().numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("K,F,metric,missing", [(64, 32, "squaredEuclidean", 0.0), (100, 33, "euclidean", 0.02),
                                                (256, 128, "squaredEuclidean", 0.005), (17, 7, "euclidean", 0.1)])
def test_cluster_mfma_on_gpu(gpu, K, F, metric, missing):
    from flink_jpmml_amd.runtime.plans import compile_plan

    c = CompiledPmml.from_string(kmeans_pmml(K, F, weighted=True, metric=metric, seed=K))
    plan = compile_plan(c, gpu, cluster_variant="mfma")
    assert plan.variant == "mfma"
    X = stream_matrix(50_000, F, seed=F, missing_rate=missing)
    s, v = _gpu_np(plan, X)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all()
    assert (s[v] == ref[v]).mean() > 0.999
    miss = np.isnan(X).any(axis=1) & v
    if miss.any():  # exact fallback rows agree with the VALU kernel bit for bit
        valu = compile_plan(c, gpu, cluster_variant="valu")
        s2, v2 = _gpu_np(valu, X[miss])
        assert (v2 == v[miss]).all() and (s2 == s[miss]).all()


@pytest.mark.gpu
def test_cluster_variant_auto(gpu):
    from flink_jpmml_amd.runtime.plans import compile_plan

    big = compile_plan(CompiledPmml.from_string(kmeans_pmml(64, 16)), gpu)
    small = compile_plan(CompiledPmml.from_string(kmeans_pmml(4, 16)), gpu)
    city = compile_plan(CompiledPmml.from_string(kmeans_pmml(64, 16, metric="cityBlock")), gpu)
    assert (big.variant, small.variant, city.variant) == ("mfma", "valu", "valu")
