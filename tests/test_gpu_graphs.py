"""HIP-graph replay of multi-kernel plans for small micro-batches (runtime/graphs.py): the
streaming engine with ``graph_max_rows`` set must produce exactly what kernel-by-kernel launches
produce, over padded row buckets, zero-copy host outputs and device mirrors."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _models():
    from flink_jpmml_amd.bench.synth import mlp_pmml, segmented_pmml, svm_pmml

    yield "gemm_mlp", mlp_pmml(n_features=24, hidden=(512, 384)), dict(mlp_impl="gemm")
    yield "segmented", segmented_pmml("median", False, n_segments=5, seed=7), {}
    yield "svm_gemm", svm_pmml(n_features=12, n_sv=80, seed=3, n_classes=5), dict(svm_impl="gemm")


@pytest.mark.parametrize("name", ["segmented", "gemm_mlp", "svm_gemm"])
@pytest.mark.parametrize("direct", [True, False])
def test_graph_replay_matches_eager(gpu, name, direct):
    import torch

    from flink_jpmml_amd.api.batch import RecordBatch
    from flink_jpmml_amd.bench.synth import stream_matrix
    from flink_jpmml_amd.runtime.compiled import CompiledPmml
    from flink_jpmml_amd.runtime.engine import StreamingScorer

    txt, opts = next((t, o) for n, t, o in _models() if n == name)
    c = CompiledPmml.from_string(txt)
    plan = c.plan(gpu, **opts)
    assert getattr(plan, "graph_small_batches", False)
    graphed = StreamingScorer(plan, micro_batch=4096, graph_max_rows=4096, direct_host_output=direct)
    eager = StreamingScorer(plan, micro_batch=4096, graph_max_rows=0, direct_host_output=direct)
    assert graphed._graphs is not None and eager._graphs is None
    for n in (1, 100, 300, 4096, 9000):  # buckets 256 / 512 / 4096, and a batch split in micro-batches
        X = stream_matrix(n, c.n_features, seed=n, missing_rate=0.02)
        rb = RecordBatch(torch.from_numpy(X).pin_memory())
        a = graphed.submit_batch(rb, keep_device=True)
        b = eager.submit_batch(rb, keep_device=True)
        np.testing.assert_array_equal(a.valid, b.valid)
        if name == "segmented":  # our kernels: identical at any padded size
            np.testing.assert_array_equal(a.scores[a.valid], b.scores[b.valid])
        elif name == "gemm_mlp":  # library GEMMs pick shape-dependent kernels: last-bit differences
            np.testing.assert_allclose(a.scores[a.valid], b.scores[b.valid], rtol=1e-5, atol=1e-6)
        else:  # SVM votes on shape-dependent GEMM decision values: near-threshold flips only
            assert (a.scores[a.valid] == b.scores[b.valid]).mean() > 0.995
        np.testing.assert_array_equal(a.device_out[0].cpu().numpy()[a.valid], a.scores[a.valid])
    assert graphed._graphs.replays > 0 and not graphed._graphs._failed
    ref, vref = c.score_matrix_oracle(X)
    assert (a.valid == vref).all()
