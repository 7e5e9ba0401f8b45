"""A DataField's explicit missing value (``<Value value="-999" property="missing"/>``, the usual
sentinel of exported numeric columns) on the device: ``build_field_prep`` lowers ONE numeric,
fp32-exact sentinel into the FieldPrep record (``FP_MISSING_VALUE``, compared in ``prep_value``
before every other treatment, as ``pmml/fields.py::prepare_matrix`` does); several sentinels and
invalid-value lists (``property="invalid"``) go into a per-field value table appended to the
FieldPrep buffer (``FP_VALUE_LIST``, round 6); string-field lists and members fp32 cannot hold
stay host-only (``NotLowerable``, never a plan that ignores them).
CPU: the lowering decisions; GPU: trees, regression, SVM, k-means and networks (through their
prepare pass) vs the float64 oracle on inputs that carry the sentinel, with and without a
missingValueReplacement. Also numeric categorical valid-value lists (label-encoded categories):
a contiguous integer run lowers to "integral and inside [min, max]", a sparse set within 64
consecutive integers to a bit mask (``FP_VALUE_MASK``), under every invalidValueTreatment; other
sets stay host-only."""

import re

import numpy as np
import pytest

from flink_jpmml_amd.runtime.compiled import CompiledPmml

SENT = -999.0


def _with_sentinel(txt: str, field: str = "f1", values=("-999",), prop: str = "missing") -> str:
    child = "".join(f'<Value value="{v}" property="{prop}"/>' for v in values)
    out, n = re.subn(rf'(<DataField name="{field}"[^>]*?)\s*/>', rf'\1>{child}</DataField>', txt, count=1)
    assert n == 1
    return out


def _with_replacement(txt: str, field: str = "f1", value: str = "0.3") -> str:
    out = txt.replace(f'<MiningField name="{field}"/>',
                      f'<MiningField name="{field}" missingValueReplacement="{value}"/>', 1)
    assert out != txt
    return out


def _models():
    from flink_jpmml_amd.bench.synth import (gbdt_pmml, kmeans_pmml, mlp_pmml, random_forest_pmml,
                                             regression_design_pmml, svm_pmml)

    return {
        "gbdt": (gbdt_pmml(n_trees=20, depth=5, n_features=6, seed=1), {}),
        "rf": (random_forest_pmml(n_trees=12, depth=5, n_features=6, n_classes=3, seed=2), {}),
        "regression": (regression_design_pmml(n_features=6, seed=3), {}),  # + categorical "color" column
        "svm": (svm_pmml(n_features=6, n_sv=40, seed=4), {}),
        "kmeans": (kmeans_pmml(n_clusters=9, n_features=6, seed=5), {}),
        "mlp": (mlp_pmml(n_features=6, hidden=(16,), seed=6), dict(precision="fp32")),
    }


MODELS = _models()


def test_sentinel_lowers_into_field_prep():
    from flink_jpmml_amd.runtime.plans import FP_HAS_MISSING_REPL, FP_MISSING_VALUE, build_field_prep

    txt = _with_replacement(_with_sentinel(MODELS["gbdt"][0]))
    c = CompiledPmml.from_string(txt)
    names = [f"f{j}" for j in range(6)]
    raw, any_prep = build_field_prep(c, names)
    assert any_prep
    assert raw[1, 0] & FP_MISSING_VALUE and raw[1, 0] & FP_HAS_MISSING_REPL
    assert raw[1:2, 7].view(np.float32)[0] == np.float32(SENT)
    assert not any(raw[j, 0] & FP_MISSING_VALUE for j in (0, 2, 3, 4, 5))


@pytest.mark.parametrize("kind", ["not-fp32", "invalid-not-fp32"])
def test_value_lists_fp32_cannot_hold_stay_host_only(kind):
    from flink_jpmml_amd.runtime.plans import NotLowerable, build_field_prep

    base = MODELS["gbdt"][0]
    txt = {"not-fp32": _with_sentinel(base, values=("0.1",)),
           "invalid-not-fp32": _with_sentinel(base, values=("-999", "0.1"), prop="invalid")}[kind]
    c = CompiledPmml.from_string(txt)
    with pytest.raises(NotLowerable):
        build_field_prep(c, [f"f{j}" for j in range(6)])


def _with_lists(txt: str, field: str = "f1", missing=("-999", "-1"), invalid=("7", "0.5")) -> str:
    child = "".join(f'<Value value="{v}" property="missing"/>' for v in missing) + \
        "".join(f'<Value value="{v}" property="invalid"/>' for v in invalid)
    out, n = re.subn(rf'(<DataField name="{field}"[^>]*?)\s*/>', rf'\1>{child}</DataField>', txt, count=1)
    assert n == 1
    return out


@pytest.mark.parametrize("treat", ["returnInvalid", "asMissing", "asIs", "asValue"])
def test_value_lists_lower_into_a_field_table(treat):
    """Several sentinels and an invalid list: FP_VALUE_LIST with the values in a table after the
    records, found through the pad word's relative offset; a line-for-line model of prep_value
    over that buffer equals the oracle's prepare on every value."""
    from flink_jpmml_amd.runtime.plans import FP_VALUE_LIST, build_field_prep

    txt = _with_lists(MODELS["gbdt"][0])
    extra = ' invalidValueReplacement="0.25"' if treat == "asValue" else ""
    txt = txt.replace('<MiningField name="f1"/>', f'<MiningField name="f1" invalidValueTreatment="{treat}"{extra}/>', 1)
    c = CompiledPmml.from_string(txt)
    names = [f"f{j}" for j in range(6)]
    raw, any_prep = build_field_prep(c, names)
    assert any_prep and raw.shape[0] > 6 and raw[1, 0] & FP_VALUE_LIST
    w = int(raw[1, 7])
    off, nm, ni = w & 0xFFFF, (w >> 16) & 0xFF, w >> 24
    flat = raw.reshape(-1).view(np.float32)
    vals = flat[1 * 8 + off: 1 * 8 + off + nm + ni]
    assert list(vals[:nm]) == [-999.0, -1.0] and list(vals[nm:]) == [7.0, 0.5]
    x = np.array([-999.0, -1.0, 7.0, 0.5, 3.0, np.nan, 0.75])
    X = np.zeros((len(x), 6))
    X[:, 1] = x
    P, ok = c.prepare(X)
    for i, xv in enumerate(x.astype(np.float32)):
        miss = bool(np.isnan(xv)) or bool(np.any(vals[:nm] == xv))
        inv = (not miss) and bool(np.any(vals[nm:] == xv))
        if inv and treat == "returnInvalid":
            assert not ok[i]
        elif inv and treat == "asMissing" or miss:
            assert np.isnan(P[i, 1]) and ok[i]
        elif inv and treat == "asValue":
            assert P[i, 1] == 0.25
        else:
            assert P[i, 1] == x[i] and ok[i]


def test_string_field_lists_are_text_level_like_the_matrix_oracle():
    """A string field's missing / invalid Value lists are matched as text by the ingest; on the
    numeric (vocabulary-code) matrix the oracle's prepare_matrix ignores them — so does the
    FieldPrep table (no flag), and the device and oracle agree."""
    from flink_jpmml_amd.runtime.plans import FP_VALUE_LIST, build_field_prep

    txt = MODELS["regression"][0]
    m = re.search(r'<DataField name="(\w+)" optype="categorical" dataType="string">', txt)
    assert m
    txt2 = txt.replace(m.group(0), m.group(0) + '<Value value="NA" property="missing"/>'
                       '<Value value="zzz" property="invalid"/>', 1)
    c, c2 = CompiledPmml.from_string(txt), CompiledPmml.from_string(txt2)
    raw, _ = build_field_prep(c2, c2.active_fields)
    j = c2.active_fields.index(m.group(1))
    assert not raw[j, 0] & FP_VALUE_LIST
    X = _inputs(300, codes=True)
    s1, v1 = c.score_matrix_oracle(X)
    s2, v2 = c2.score_matrix_oracle(X)
    assert (v1 == v2).all()
    np.testing.assert_array_equal(s1[v1], s2[v2])


@pytest.mark.parametrize("values,flagged", [(("NA",), False), (("NA", "-999", "?"), True)])
def test_non_numeric_missing_values_are_ignored_on_numeric_fields(values, flagged):
    """A numeric matrix cannot hold "NA": like the oracle's prepare_matrix, only the numeric
    sentinel takes part."""
    from flink_jpmml_amd.runtime.plans import FP_MISSING_VALUE, build_field_prep

    c = CompiledPmml.from_string(_with_sentinel(MODELS["gbdt"][0], values=values))
    raw, _ = build_field_prep(c, [f"f{j}" for j in range(6)])
    assert bool(raw[1, 0] & FP_MISSING_VALUE) == flagged
    X = _inputs(400)
    ref, vref = c.score_matrix_oracle(X)
    c0 = CompiledPmml.from_string(_with_sentinel(MODELS["gbdt"][0], values=("-999",) if flagged else ()))
    ref0, vref0 = c0.score_matrix_oracle(X)
    assert (vref == vref0).all()
    np.testing.assert_array_equal(ref[vref], ref0[vref0])


@pytest.mark.parametrize("name", list(MODELS))
def test_every_family_lowers_with_a_sentinel(name):
    from flink_jpmml_amd.runtime.plans import lowering_dry_run

    txt, opts = MODELS[name]
    c = CompiledPmml.from_string(_with_sentinel(txt))
    with lowering_dry_run():
        plan = c.plan("cpu", **opts)
    preps = [getattr(plan, "prep", None), getattr(getattr(plan, "inner", None), "prep", None)]
    assert any(p is not None for p in preps), type(plan).__name__


def test_oracle_treats_the_sentinel_as_missing():
    base = MODELS["gbdt"][0]
    c0, c1 = CompiledPmml.from_string(base), CompiledPmml.from_string(_with_sentinel(base))
    X = _inputs(500)
    Xn = X.copy()
    Xn[Xn[:, 1] == SENT, 1] = np.nan
    s1, v1 = c1.score_matrix_oracle(X)
    s0, v0 = c0.score_matrix_oracle(Xn)
    assert (v1 == v0).all()
    np.testing.assert_array_equal(s1[v1], s0[v0])


def _inputs(n: int, codes: bool = False) -> np.ndarray:
    from flink_jpmml_amd.bench.synth import stream_matrix

    X = stream_matrix(n, 6, seed=11, missing_rate=0.02)
    rng = np.random.default_rng(12)
    X[rng.random(n) < 0.25, 1] = SENT
    if codes:  # the regression model's string field, as category codes
        X = np.concatenate([X, rng.integers(0, 3, (n, 1)).astype(X.dtype)], axis=1)
    return X


@pytest.mark.gpu
@pytest.mark.parametrize("repl", [False, True], ids=["missing", "replaced"])
@pytest.mark.parametrize("name", list(MODELS))
def test_sentinel_on_gpu(gpu, name, repl):
    txt, opts = MODELS[name]
    txt = _with_sentinel(txt)
    if repl:
        txt = _with_replacement(txt)
    c = CompiledPmml.from_string(txt)
    plan = c.plan(gpu, **opts)
    preps = [getattr(plan, "prep", None), getattr(getattr(plan, "inner", None), "prep", None)]
    assert any(p is not None for p in preps), f"{type(plan).__name__} lowered without a FieldPrep table"
    X = _inputs(5000, codes=name == "regression")
    s, v = plan.score(X)
    s, v = s.cpu().numpy().astype(np.float64), v.cpu().numpy().astype(bool)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all()
    assert v.any()
    if name in ("rf", "kmeans"):
        assert (s[v] == ref[v]).mean() >= 0.995
    else:
        scale = max(1.0, float(np.abs(ref[v]).max()))
        np.testing.assert_allclose(s[v], ref[v], rtol=0, atol=2e-4 * scale)


def _categorical(txt: str, values=("0", "1", "2", "3"), treat: str = "returnInvalid") -> str:
    child = "".join(f'<Value value="{v}"/>' for v in values)
    out, n = re.subn(r'<DataField name="f1"[^>]*/>',
                     f'<DataField name="f1" optype="categorical" dataType="integer">{child}</DataField>', txt, count=1)
    assert n == 1
    extra = ' invalidValueReplacement="2"' if treat == "asValue" else ""
    return out.replace('<MiningField name="f1"/>', f'<MiningField name="f1" invalidValueTreatment="{treat}"{extra}/>', 1)


def _categorical_inputs(n: int, codes: bool = False) -> np.ndarray:
    X = _inputs(n, codes)
    X[:, 1] = np.random.default_rng(13).choice([0, 1, 2, 3, 4, -1, 1.5, 50, 51, -2, np.nan], n)
    return X


def test_integer_category_run_lowers_to_interval_and_integer():
    from flink_jpmml_amd.runtime.plans import FP_HAS_INTERVAL, FP_INTEGER, FP_INVALID_AS_MISSING, build_field_prep

    c = CompiledPmml.from_string(_categorical(MODELS["gbdt"][0], values=("3", "1", "2", "0"), treat="asMissing"))
    raw, _ = build_field_prep(c, [f"f{j}" for j in range(6)])
    assert raw[1, 0] & (FP_HAS_INTERVAL | FP_INTEGER | FP_INVALID_AS_MISSING) == \
        FP_HAS_INTERVAL | FP_INTEGER | FP_INVALID_AS_MISSING
    assert list(raw[1:2, 1:3].view(np.float32)[0]) == [0.0, 3.0]


def test_sparse_integer_category_set_lowers_to_a_bit_mask():
    from flink_jpmml_amd.runtime.plans import FP_VALUE_MASK, build_field_prep

    c = CompiledPmml.from_string(_categorical(MODELS["gbdt"][0], values=("-3", "0", "2", "40", "60")))
    raw, _ = build_field_prep(c, [f"f{j}" for j in range(6)])
    assert raw[1, 0] & FP_VALUE_MASK
    assert raw[1:2, 1].view(np.float32)[0] == -3.0
    bits = int(raw[1, 5]) | (int(raw[1, 6]) << 32)
    assert bits == sum(1 << (v + 3) for v in (-3, 0, 2, 40, 60))


def _mask_model_valid(x: np.ndarray, lo: float, bits: int) -> np.ndarray:
    """Line-for-line model of prep_value's FP_VALUE_MASK test (fp32)."""
    x = x.astype(np.float32)
    d = x - np.float32(lo)
    ok = (d >= 0) & (d < 64) & (np.floor(x) == x)
    k = np.where(ok, d, 0).astype(np.uint64)
    return ok & (((np.uint64(bits) >> k) & np.uint64(1)) == 1)


def test_value_mask_model_matches_the_oracle_validity():
    values = ("-3", "0", "2", "40", "60")
    c = CompiledPmml.from_string(_categorical(MODELS["gbdt"][0], values=values))
    X = _inputs(3000)
    X[:, 1] = np.random.default_rng(5).choice([-4, -3, -2.5, 0, 1, 2, 39, 40, 60, 61, 70, np.nan], 3000)
    _, vref = c.score_matrix_oracle(X)
    bits = sum(1 << (int(v) + 3) for v in values)
    miss_elsewhere = np.isnan(X).any(axis=1) & ~np.isnan(X[:, 1])
    model = _mask_model_valid(X[:, 1], -3.0, bits) | np.isnan(X[:, 1])
    # the GBDT scores rows with other missing features too; only f1's validity decides here
    assert (vref[~miss_elsewhere] == model[~miss_elsewhere]).all()


@pytest.mark.parametrize("values", [("0", "100"), ("0.5", "1.5"), ("a", "1")])
def test_other_numeric_category_sets_stay_host_only(values):
    from flink_jpmml_amd.runtime.plans import NotLowerable, build_field_prep

    c = CompiledPmml.from_string(_categorical(MODELS["gbdt"][0], values=values))
    with pytest.raises(NotLowerable):
        build_field_prep(c, [f"f{j}" for j in range(6)])


@pytest.mark.gpu
@pytest.mark.parametrize("values", [("0", "1", "2", "3"), ("-1", "1", "3", "50")], ids=["run", "mask"])
@pytest.mark.parametrize("treat", ["returnInvalid", "asMissing", "asIs", "asValue"])
@pytest.mark.parametrize("name", ["gbdt", "svm", "mlp"])
def test_integer_categories_on_gpu(gpu, name, treat, values):
    txt, opts = MODELS[name]
    c = CompiledPmml.from_string(_categorical(txt, values=values, treat=treat))
    plan = c.plan(gpu, **opts)
    X = _categorical_inputs(4000)
    s, v = plan.score(X)
    s, v = s.cpu().numpy().astype(np.float64), v.cpu().numpy().astype(bool)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all()
    assert v.any()
    scale = max(1.0, float(np.abs(ref[v]).max()))
    np.testing.assert_allclose(s[v], ref[v], rtol=0, atol=2e-4 * scale)


@pytest.mark.gpu
@pytest.mark.parametrize("treat", ["returnInvalid", "asMissing", "asValue"])
@pytest.mark.parametrize("name", ["gbdt", "rf", "regression", "svm", "kmeans", "mlp"])
def test_value_lists_on_gpu(gpu, name, treat):
    """Several sentinels + an invalid-value list lowered into the FieldPrep value table: validity
    and scores equal the oracle with ``fallback="error"`` semantics (the plan must exist)."""
    txt, opts = MODELS[name]
    txt = _with_lists(txt, missing=("-999", "-1", "4"), invalid=("7", "0.5", "-2"))
    extra = ' invalidValueReplacement="0.25"' if treat == "asValue" else ""
    txt = txt.replace('<MiningField name="f1"/>', f'<MiningField name="f1" invalidValueTreatment="{treat}"{extra}/>', 1)
    c = CompiledPmml.from_string(txt)
    plan = c.plan(gpu, **opts)
    X = _inputs(6000, codes=name == "regression")
    rng = np.random.default_rng(21)
    X[:, 1] = np.where(rng.random(len(X)) < 0.5, rng.choice([-999.0, -1.0, 4.0, 7.0, 0.5, -2.0], len(X)), X[:, 1])
    s, v = plan.score(X)
    s, v = s.cpu().numpy().astype(np.float64), v.cpu().numpy().astype(bool)
    ref, vref = c.score_matrix_oracle(X)
    assert (v == vref).all()
    assert v.any()
    if name in ("rf", "kmeans"):
        assert (s[v] == ref[v]).mean() >= 0.995
    else:
        scale = max(1.0, float(np.abs(ref[v]).max()))
        np.testing.assert_allclose(s[v], ref[v], rtol=0, atol=2e-4 * scale)


@pytest.mark.gpu
def test_near_sentinel_input_is_missing_on_the_device_only(gpu):
    """ADVICE r5 (low), documented in docs/PARITY.md "Deliberate deviations": a float64 input within
    half an fp32 ulp of the sentinel rounds onto it in the fp32 row the kernels read, so the device
    treats it as missing while the float64 oracle keeps the value."""
    base = MODELS["gbdt"][0].replace('<DataField name="f1" optype="continuous" dataType="float"/>',
                                     '<DataField name="f1" optype="continuous" dataType="double"/>')
    assert 'name="f1" optype="continuous" dataType="double"' in base  # float fields round first (no deviation)
    txt = _with_replacement(_with_sentinel(base))
    c = CompiledPmml.from_string(txt)
    plan = c.plan(gpu)
    near = -999.00003  # |near - (-999)| < half an fp32 ulp (3.05e-5) at 999
    assert np.float32(near) == np.float32(SENT) and near != SENT
    X = _inputs(64).astype(np.float64)  # float64 records: -999.00003 is representable
    X[:, 1] = near
    Xs = X.copy()
    Xs[:, 1] = SENT
    s_near, _ = plan.score(X)
    s_sent, _ = plan.score(Xs)
    np.testing.assert_array_equal(s_near.cpu().numpy(), s_sent.cpu().numpy())  # device: missing
    P_near, _ = c.prepare(X)
    P_sent, _ = c.prepare(Xs)
    assert (P_near[:, 1] == near).all()  # oracle: -999.00003 is a value, not the sentinel
    assert (P_sent[:, 1] == 0.3).all()  # the sentinel takes the missingValueReplacement
