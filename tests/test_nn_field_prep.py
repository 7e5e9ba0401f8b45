"""NeuralNetworks whose inputs carry a MiningField / DataField treatment (missing-value
replacement, validity interval with each invalid treatment, outliers): the network kernels read
raw columns, so compile_plan must put a prepare-only derive pass in front (DerivedPlan → the
network plan on prepared inputs) — never a plan that silently skips the treatment. CPU: lowering
decisions (dry run); GPU: every treatment vs the float64 oracle on the fused, wide and library-GEMM
network plans."""

import re

import numpy as np
import pytest

from flink_jpmml_amd.bench.synth import mlp_pmml, stream_matrix
from flink_jpmml_amd.runtime.compiled import CompiledPmml


def _variants():
    base = mlp_pmml(n_features=8, hidden=(16, 12), seed=1)
    iv = r'\1><Interval closure="closedClosed" leftMargin="-1" rightMargin="1"/></DataField>'
    out = {"plain": base,
           "mvr": base.replace('<MiningField name="f0"/>', '<MiningField name="f0" missingValueReplacement="0.5"/>', 1)}
    for treat in ("asMissing", "returnInvalid", "asIs"):
        t = re.sub(r'(<DataField name="f1"[^>]*)/>', iv, base, count=1)
        out[f"interval-{treat}"] = t.replace('<MiningField name="f1"/>',
                                             f'<MiningField name="f1" invalidValueTreatment="{treat}"/>', 1)
    t = re.sub(r'(<DataField name="f2"[^>]*)/>', iv, base, count=1)
    out["interval-asValue"] = t.replace('<MiningField name="f2"/>', '<MiningField name="f2" invalidValueTreatment='
                                        '"asValue" invalidValueReplacement="0.25"/>', 1)
    out["outliers-extreme"] = base.replace('<MiningField name="f3"/>', '<MiningField name="f3" outliers='
                                           '"asExtremeValues" lowValue="-0.5" highValue="0.5"/>', 1)
    out["outliers-missing"] = base.replace('<MiningField name="f4"/>', '<MiningField name="f4" outliers='
                                           '"asMissingValues" lowValue="-1" highValue="1" missingValueReplacement="0"/>', 1)
    for k, v in out.items():
        assert k == "plain" or v != base, k
    return out


VARIANTS = _variants()


@pytest.mark.parametrize("name", list(VARIANTS))
@pytest.mark.parametrize("opts", [dict(precision="bf16"), dict(precision="fp32", mlp_impl="wide"),
                                  dict(mlp_impl="gemm")], ids=["fused", "wide", "gemm"])
def test_network_plans_get_a_prepare_pass(name, opts):
    from flink_jpmml_amd.runtime.derive import DerivedPlan
    from flink_jpmml_amd.runtime.plans import lowering_dry_run

    c = CompiledPmml.from_string(VARIANTS[name])
    with lowering_dry_run():
        plan = c.plan("cpu", **opts)
    if name == "plain":
        assert not isinstance(plan, DerivedPlan) and plan.prep is None
    else:
        assert isinstance(plan, DerivedPlan) and plan.inner.prep is None and plan.prep is not None


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(VARIANTS))
@pytest.mark.parametrize("opts", [dict(precision="bf16"), dict(precision="fp32", mlp_impl="wide"),
                                  dict(mlp_impl="gemm")], ids=["fused", "wide", "gemm"])
def test_network_field_treatments_on_gpu(gpu, name, opts):
    c = CompiledPmml.from_string(VARIANTS[name])
    plan = c.plan(gpu, **opts)
    X = stream_matrix(6000, 8, seed=3, missing_rate=0.05) * 1.5  # values outside [-1, 1] and missing
    s, v = plan.score(X)
    s, v = s.cpu().numpy().astype(np.float64), v.cpu().numpy().astype(bool)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all()
    tol = 3e-2 if opts.get("precision") == "bf16" else 1e-4
    scale = max(1.0, float(np.abs(ref[v]).max())) if v.any() else 1.0
    assert np.abs(s[v] - ref[v]).max() < tol * scale
