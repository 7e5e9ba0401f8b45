"""Randomized MiningField / DataField treatments on the device vs the float64 oracle: every field
of a random model (GBDT, random forest, SVM, k-means, MLP) draws a random combination of
missingValueReplacement, a validity Interval (each closure) with each invalidValueTreatment,
outliers (asExtremeValues / asMissingValues), an explicit missing-value sentinel and an integer
dataType; the inputs hit every branch (missing, sentinel, outside the interval, outliers,
non-integral). The kernels apply all of it in ``common.h::prep_value`` (networks through their
prepare pass): validity must equal the oracle's row for row, scores within fp32. CPU part: the
per-record and columnar oracles agree on every drawn row, and every drawn document lowers (no
``NotLowerable``)."""

import re

import numpy as np
import pytest

from tests._suite import gpu_seeds

from flink_jpmml_amd.runtime.compiled import CompiledPmml

F = 6
SENT = -999.0


def _model(kind: str, seed: int) -> tuple:
    from flink_jpmml_amd.bench.synth import gbdt_pmml, kmeans_pmml, mlp_pmml, random_forest_pmml, svm_pmml

    if kind == "gbdt":
        return gbdt_pmml(n_trees=24, depth=5, n_features=F, seed=seed), {}, False
    if kind == "rf":
        return random_forest_pmml(n_trees=16, depth=5, n_features=F, n_classes=3, seed=seed), {}, True
    if kind == "svm":
        return svm_pmml(n_features=F, n_sv=48, seed=seed), {}, False
    if kind == "kmeans":
        return kmeans_pmml(n_clusters=7, n_features=F, seed=seed), {}, True
    return mlp_pmml(n_features=F, hidden=(16, 8), seed=seed), dict(precision="fp32"), False


def _treat(txt: str, rng: np.random.Generator) -> tuple:
    """Random treatments per field; returns (document, per-field sentinel flags, integer flags)."""
    sentinel, integer = [], []
    for j in range(F):
        name = f"f{j}"
        attrs, children = [], []
        has_iv = rng.random() < 0.5
        integ = rng.random() < 0.15 and not has_iv
        if rng.random() < 0.4:  # an integer field's replacement is an integer (else the document is invalid)
            attrs.append(f'missingValueReplacement="{int(rng.integers(-1, 2)) if integ else round(rng.uniform(-1, 1), 3)}"')
        if has_iv:
            lo = rng.uniform(-1.5, -0.2)
            hi = rng.uniform(0.2, 1.5)
            closure = rng.choice(["closedClosed", "openOpen", "closedOpen", "openClosed"])
            children.append(f'<Interval closure="{closure}" leftMargin="{lo:.3f}" rightMargin="{hi:.3f}"/>')
            treat = rng.choice(["returnInvalid", "asMissing", "asIs", "asValue"])
            attrs.append(f'invalidValueTreatment="{treat}"')
            if treat == "asValue":
                attrs.append(f'invalidValueReplacement="{rng.uniform(-0.5, 0.5):.3f}"')
        if rng.random() < 0.35:
            kind = rng.choice(["asExtremeValues", "asMissingValues"])
            attrs.append(f'outliers="{kind}" lowValue="{rng.uniform(-2, -0.5):.3f}" highValue="{rng.uniform(0.5, 2):.3f}"')
        sent = rng.random() < 0.3
        if sent:
            children.insert(0, f'<Value value="{SENT:g}" property="missing"/>')
        sentinel.append(sent)
        integer.append(integ)
        if children or integ:
            dtype = ' dataType="integer"' if integ else ""
            pat = rf'<DataField name="{name}" optype="continuous" dataType="(\w+)"\s*/>'
            m = re.search(pat, txt)
            assert m is not None, name
            dt = dtype or f' dataType="{m.group(1)}"'
            txt = txt[:m.start()] + (f'<DataField name="{name}" optype="continuous"{dt}>{"".join(children)}'
                                     '</DataField>') + txt[m.end():]
        if attrs:
            old = f'<MiningField name="{name}"/>'
            assert old in txt, name
            txt = txt.replace(old, f'<MiningField name="{name}" {" ".join(attrs)}/>', 1)
    return txt, sentinel, integer


def _inputs(n: int, sentinel, integer, seed: int) -> np.ndarray:
    from flink_jpmml_amd.bench.synth import stream_matrix

    rng = np.random.default_rng(seed)
    X = stream_matrix(n, F, seed=seed, missing_rate=0.02) * 1.4
    for j in range(F):
        if sentinel[j]:
            X[rng.random(n) < 0.1, j] = SENT
        if integer[j]:
            r = rng.random(n) < 0.7
            X[r, j] = np.round(X[r, j])
    return X


KINDS = ["gbdt", "rf", "svm", "kmeans", "mlp"]


def _case(seed: int):
    rng = np.random.default_rng(9100 + seed)
    kind = KINDS[seed % len(KINDS)]
    txt, opts, label = _model(kind, seed)
    txt, sentinel, integer = _treat(txt, rng)
    return kind, txt, opts, label, sentinel, integer


@pytest.mark.parametrize("seed", range(40))
def test_record_and_matrix_oracles_agree(seed):
    """The per-record oracle (``FieldSchema.prepare_value``, the reference's record path) and the
    columnar one (``prepare_matrix``, which the device is checked against) prepare every drawn
    row identically — this fuzz found two splits between them: outliers applied to invalid asIs /
    asValue values on the matrix path, and "-999.0" not matching a "-999" sentinel per record."""
    kind, txt, opts, _, sentinel, integer = _case(seed)
    c = CompiledPmml.from_string(txt)
    X = _inputs(200, sentinel, integer, seed)
    P, ok = c.prepare(X)
    for r in range(len(X)):
        vals = []
        try:
            for j, name in enumerate(c.active_fields):
                raw = None if np.isnan(X[r, j]) else float(X[r, j])
                vals.append(c.schema.prepare_value(name, raw, c.mining_fields.get(name)))
        except Exception:  # noqa: BLE001 - InvalidValue: the record scores EmptyScore
            assert not ok[r], (kind, r)
            continue
        assert ok[r], (kind, r)
        np.testing.assert_allclose(np.array(vals), P[r], rtol=0, atol=1e-6, equal_nan=True, err_msg=f"{kind} {r}")


@pytest.mark.parametrize("seed", range(10))
def test_random_treatments_lower(seed):
    from flink_jpmml_amd.runtime.plans import lowering_dry_run

    kind, txt, opts, _, _, _ = _case(seed)
    c = CompiledPmml.from_string(txt)
    with lowering_dry_run():
        c.plan("cpu", **opts)  # raises NotLowerable if a treatment were host-only


@pytest.mark.gpu
@pytest.mark.parametrize("seed", gpu_seeds(40, 12))
def test_random_treatments_on_gpu(gpu, seed):
    kind, txt, opts, label, sentinel, integer = _case(seed)
    c = CompiledPmml.from_string(txt)
    plan = c.plan(gpu, **opts)
    X = _inputs(4000, sentinel, integer, seed)
    s, v = plan.score(X)
    s, v = s.cpu().numpy().astype(np.float64), v.cpu().numpy().astype(bool)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all(), f"{kind}: validity differs on {(v != vref).sum()} rows"
    if not v.any():
        return
    if label:
        assert (s[v] == ref[v]).mean() >= 0.99
    else:
        scale = max(1.0, float(np.abs(ref[v]).max()))
        np.testing.assert_allclose(s[v], ref[v], rtol=0, atol=2e-4 * scale)
