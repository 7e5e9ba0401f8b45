"""Synthetic PMML model + data generators for the benchmark configs of ``BASELINE.json``.

No network, no checkpoints: every model is random-initialised with the *structure* of the named
exporter and written as a PMML document, then loaded back through the normal parser, so the
benchmark measures the real load → compile → score path.

* :func:`gbdt_pmml` — XGBoost-style (JPMML-XGBoost layout) gradient-boosted trees:
  ``MiningModel(sum)`` of binary ``TreeModel``s with ``defaultChild`` missing routing, float
  fields, base score in ``Targets/@rescaleConstant``; ``objective="binary"`` adds the
  ``modelChain`` → ``RegressionModel(logit)`` calibrator (config 5).
* :func:`random_forest_pmml` — scikit-learn-style ``majorityVote`` forest (config 3).
* :func:`iris_logistic_pmml` — multinomial logistic regression on Iris (config 1).
* :func:`mlp_pmml` — 3-layer ``NeuralNetwork`` (config 4).
* :func:`svm_pmml` — RBF ``SupportVectorMachineModel``.
* :func:`stream_matrix` — the synthetic record stream (fp32, optional missing values).
"""

from __future__ import annotations

import io
from typing import List, Optional, Tuple

import numpy as np

NS = "http://www.dmg.org/PMML-4_4"


def _header(out: io.StringIO, desc: str) -> None:
    out.write(f'<?xml version="1.0" encoding="UTF-8"?>\n<PMML version="4.4" xmlns="{NS}">\n')
    out.write(f' <Header description="{desc}"><Application name="flink_jpmml_amd.bench.synth" version="1"/></Header>\n')


def _fnum(x: float) -> str:
    return repr(float(np.float32(x)))


class _TreeGen:
    def __init__(self, rng: np.random.Generator, n_features: int, depth: int, p_split: float,
                 thresholds: np.ndarray, field_fmt: str = "f{}"):
        self.rng = rng
        self.F = n_features
        self.depth = depth
        self.p_split = p_split
        self.thr = thresholds
        self.fmt = field_fmt
        self.next_id = 0

    def nid(self) -> int:
        self.next_id += 1
        return self.next_id

    def write(self, out: io.StringIO, depth: int, pred: str, leaf_fn, indent: str, force_split: bool = False) -> None:
        my = self.nid()
        split = depth < self.depth and (force_split or self.rng.random() < self.p_split)
        if not split:
            out.write(f'{indent}<Node id="{my}" score="{leaf_fn()}">{pred}</Node>\n')
            return
        f = int(self.rng.integers(self.F))
        t = _fnum(self.thr[f, int(self.rng.integers(self.thr.shape[1]))])
        left_id = self.next_id + 1  # ids are assigned depth-first: the left child is next
        go_left = bool(self.rng.random() < 0.5)
        # write children into a buffer first to learn the right child's id
        buf = io.StringIO()
        name = self.fmt.format(f)
        self.write(buf, depth + 1, f'<SimplePredicate field="{name}" operator="lessThan" value="{t}"/>', leaf_fn,
                   indent + " ")
        right_id = self.next_id + 1
        self.write(buf, depth + 1, f'<SimplePredicate field="{name}" operator="greaterOrEqual" value="{t}"/>',
                   leaf_fn, indent + " ")
        dflt = left_id if go_left else right_id
        out.write(f'{indent}<Node id="{my}" defaultChild="{dflt}">{pred}\n')
        out.write(buf.getvalue())
        out.write(f'{indent}</Node>\n')


def _data_dictionary(out: io.StringIO, F: int, target: str, target_type: str = "double",
                     categories: Optional[List[str]] = None) -> None:
    out.write(f' <DataDictionary numberOfFields="{F + 1}">\n')
    for j in range(F):
        out.write(f'  <DataField name="f{j}" optype="continuous" dataType="float"/>\n')
    if categories is None:
        out.write(f'  <DataField name="{target}" optype="continuous" dataType="{target_type}"/>\n')
    else:
        out.write(f'  <DataField name="{target}" optype="categorical" dataType="{target_type}">\n')
        for c in categories:
            out.write(f'   <Value value="{c}"/>\n')
        out.write('  </DataField>\n')
    out.write(' </DataDictionary>\n')


def _mining_schema(out: io.StringIO, F: int, target: Optional[str], indent: str = "  ") -> None:
    out.write(f'{indent}<MiningSchema>\n')
    if target is not None:
        out.write(f'{indent} <MiningField name="{target}" usageType="target"/>\n')
    for j in range(F):
        out.write(f'{indent} <MiningField name="f{j}"/>\n')
    out.write(f'{indent}</MiningSchema>\n')


def gbdt_pmml(n_trees: int = 1000, depth: int = 6, n_features: int = 32, seed: int = 0,
              objective: str = "regression", p_split: float = 0.9, learning_rate: float = 0.1,
              base_score: float = 0.5, float_casts: bool = False, missing_strategy: str = "defaultChild",
              n_classes: int = 3, scaled: bool = False) -> str:
    """XGBoost-style GBDT PMML: regression, ``binary`` (binary:logistic chain) or ``multiclass``
    (multi:softprob — ``n_classes`` chained ensembles of ``n_trees`` each + a softmax
    RegressionModel over their ``xgbValue(k)`` outputs). ``float_casts`` adds the
    ``float(fj)`` ``LocalTransformations`` casts that pipeline exporters (sklearn2pmml) emit, with
    every split on the cast field. ``scaled`` splits on monotone derived fields ``d(fj)`` instead:
    StandardScaler-style ``(x - mu) / sd``, increasing and clamped ``NormContinuous``, and a
    decreasing ``(c - x) * k`` (the sklearn2pmml preprocessing shapes)."""
    rng = np.random.default_rng(seed)
    thresholds = np.sort(rng.standard_normal((n_features, 64)).astype(np.float32), axis=1)
    out = io.StringIO()
    _header(out, f"synthetic GBDT {n_trees} trees depth {depth} ({objective})")
    binary = objective == "binary"
    multi = objective == "multiclass"
    cats = [str(k) for k in range(n_classes)] if multi else ["0", "1"]
    _data_dictionary(out, n_features, "y", "integer" if binary or multi else "double", cats if binary or multi else None)
    fmt = "d(f{})" if scaled else ("float(f{})" if float_casts else "f{}")

    def leaf() -> str:
        return _fnum(learning_rate * rng.standard_normal())

    def scalers(indent: str) -> None:
        out.write(f'{indent}<LocalTransformations>\n')
        for j in range(n_features):
            kind = j % 4
            if kind == 0:
                ex = (f'<Apply function="/"><Apply function="-"><FieldRef field="f{j}"/><Constant>{0.1 * j:.3f}'
                      f'</Constant></Apply><Constant>1.25</Constant></Apply>')
            elif kind == 1:
                ex = (f'<NormContinuous field="f{j}"><LinearNorm orig="-2" norm="-1.5"/><LinearNorm orig="0" '
                      f'norm="0.25"/><LinearNorm orig="1.5" norm="1"/></NormContinuous>')
            elif kind == 2:
                ex = f'<Apply function="*"><Apply function="-"><Constant>0.5</Constant><FieldRef field="f{j}"/></Apply><Constant>0.8</Constant></Apply>'
            else:
                ex = (f'<NormContinuous field="f{j}" outliers="asExtremeValues"><LinearNorm orig="-1" norm="-1"/>'
                      f'<LinearNorm orig="1" norm="1"/></NormContinuous>')
            out.write(f'{indent} <DerivedField name="d(f{j})" optype="continuous" dataType="double">{ex}</DerivedField>\n')
        out.write(f'{indent}</LocalTransformations>\n')

    def casts(indent: str) -> None:
        if scaled:
            scalers(indent)
            return
        if not float_casts:
            return
        out.write(f'{indent}<LocalTransformations>\n')
        for j in range(n_features):
            out.write(f'{indent} <DerivedField name="float(f{j})" optype="continuous" dataType="float">'
                      f'<FieldRef field="f{j}"/></DerivedField>\n')
        out.write(f'{indent}</LocalTransformations>\n')

    def trees_model(indent: str, target_in_schema: bool, rescale: float, out_name: str = "xgbValue") -> None:
        out.write(f'{indent}<MiningModel functionName="regression">\n')
        _mining_schema(out, n_features, None if not target_in_schema else "y", indent + " ")
        if binary or multi:
            out.write(f'{indent} <Output><OutputField name="{out_name}" optype="continuous" dataType="float" '
                      f'isFinalResult="false"/></Output>\n')
        out.write(f'{indent} <Targets><Target rescaleConstant="{_fnum(rescale)}"/></Targets>\n')
        casts(indent + " ")
        out.write(f'{indent} <Segmentation multipleModelMethod="sum">\n')
        for t in range(n_trees):
            g = _TreeGen(rng, n_features, depth, p_split, thresholds, fmt)
            out.write(f'{indent}  <Segment id="{t + 1}"><True/>\n')
            out.write(f'{indent}   <TreeModel functionName="regression" missingValueStrategy="{missing_strategy}" '
                      f'noTrueChildStrategy="returnLastPrediction" splitCharacteristic="binarySplit">\n')
            _mining_schema(out, n_features, None, indent + "    ")
            g.write(out, 0, "<True/>", leaf, indent + "    ", force_split=True)
            out.write(f'{indent}   </TreeModel>\n{indent}  </Segment>\n')
        out.write(f'{indent} </Segmentation>\n{indent}</MiningModel>\n')

    if not binary and not multi:
        out.write(' <MiningModel functionName="regression" algorithmName="XGBoost (GBTree)">\n')
        _mining_schema(out, n_features, "y", "  ")
        out.write(f'  <Targets><Target field="y" rescaleConstant="{_fnum(base_score)}"/></Targets>\n')
        casts("  ")
        out.write('  <Segmentation multipleModelMethod="sum">\n')
        for t in range(n_trees):
            g = _TreeGen(rng, n_features, depth, p_split, thresholds, fmt)
            out.write(f'   <Segment id="{t + 1}"><True/>\n')
            out.write(f'    <TreeModel functionName="regression" missingValueStrategy="{missing_strategy}" '
                      'noTrueChildStrategy="returnLastPrediction" splitCharacteristic="binarySplit">\n')
            _mining_schema(out, n_features, None, "     ")
            g.write(out, 0, "<True/>", leaf, "     ", force_split=True)
            out.write('    </TreeModel>\n   </Segment>\n')
        out.write('  </Segmentation>\n </MiningModel>\n</PMML>\n')
        return out.getvalue()
    out.write(' <MiningModel functionName="classification" algorithmName="XGBoost (GBTree)">\n')
    _mining_schema(out, n_features, "y", "  ")
    out.write('  <Segmentation multipleModelMethod="modelChain">\n')
    if multi:
        for k in range(n_classes):
            out.write(f'   <Segment id="{k + 1}"><True/>\n')
            trees_model("    ", False, 0.0, f"xgbValue({k})")
            out.write('   </Segment>\n')
        out.write(f'   <Segment id="{n_classes + 1}"><True/>\n')
        out.write('    <RegressionModel functionName="classification" normalizationMethod="softmax">\n')
        out.write('     <MiningSchema><MiningField name="y" usageType="target"/>'
                  + "".join(f'<MiningField name="xgbValue({k})"/>' for k in range(n_classes)) + '</MiningSchema>\n')
        for k in range(n_classes):
            out.write(f'     <RegressionTable intercept="{_fnum(0.1 * k)}" targetCategory="{k}">'
                      f'<NumericPredictor name="xgbValue({k})" coefficient="1.0"/></RegressionTable>\n')
        out.write('    </RegressionModel>\n   </Segment>\n  </Segmentation>\n </MiningModel>\n</PMML>\n')
        return out.getvalue()
    out.write('   <Segment id="1"><True/>\n')
    trees_model("    ", False, float(np.log(base_score / (1 - base_score))))
    out.write('   </Segment>\n   <Segment id="2"><True/>\n')
    out.write('    <RegressionModel functionName="classification" normalizationMethod="logit">\n')
    out.write('     <MiningSchema><MiningField name="y" usageType="target"/>'
              '<MiningField name="xgbValue"/></MiningSchema>\n')
    out.write('     <RegressionTable intercept="0.0" targetCategory="1">'
              '<NumericPredictor name="xgbValue" coefficient="1.0"/></RegressionTable>\n')
    out.write('     <RegressionTable intercept="0.0" targetCategory="0"/>\n')
    out.write('    </RegressionModel>\n   </Segment>\n  </Segmentation>\n </MiningModel>\n</PMML>\n')
    return out.getvalue()


def random_forest_pmml(n_trees: int = 500, depth: int = 8, n_features: int = 32, n_classes: int = 3,
                       seed: int = 0, p_split: float = 0.85, missing_strategy: str = "defaultChild") -> str:
    """scikit-learn-style majority-vote random forest (classification trees). ``missing_strategy``
    ``"nullPrediction"`` is what sklearn2pmml exports: a missing split value voids the tree."""
    rng = np.random.default_rng(seed)
    thresholds = np.sort(rng.standard_normal((n_features, 64)).astype(np.float32), axis=1)
    cats = [str(c) for c in range(n_classes)]
    out = io.StringIO()
    _header(out, f"synthetic random forest {n_trees} trees depth {depth}")
    _data_dictionary(out, n_features, "y", "integer", cats)
    out.write(' <MiningModel functionName="classification" algorithmName="sklearn RandomForest">\n')
    _mining_schema(out, n_features, "y", "  ")
    out.write('  <Segmentation multipleModelMethod="majorityVote">\n')
    for t in range(n_trees):
        g = _TreeGen(rng, n_features, depth, p_split, thresholds)
        out.write(f'   <Segment id="{t + 1}"><True/>\n')
        out.write(f'    <TreeModel functionName="classification" missingValueStrategy="{missing_strategy}" '
                  'splitCharacteristic="binarySplit">\n')
        _mining_schema(out, n_features, "y", "     ")
        g.write(out, 0, "<True/>", lambda: cats[int(rng.integers(n_classes))], "     ", force_split=True)
        out.write('    </TreeModel>\n   </Segment>\n')
    out.write('  </Segmentation>\n </MiningModel>\n</PMML>\n')
    return out.getvalue()


def iris_logistic_pmml() -> str:
    """Multinomial logistic regression on the four Iris features (softmax over 3 tables)."""
    fields = ["sepal_length", "sepal_width", "petal_length", "petal_width"]
    coefs = {
        "Iris-setosa": (9.85, [-0.42, 0.97, -2.52, -1.08]),
        "Iris-versicolor": (2.24, [0.53, -0.32, -0.21, -0.94]),
        "Iris-virginica": (-12.09, [-0.11, -0.65, 2.73, 2.02]),
    }
    out = io.StringIO()
    _header(out, "Iris multinomial logistic regression")
    out.write(' <DataDictionary numberOfFields="5">\n')
    for f in fields:
        out.write(f'  <DataField name="{f}" optype="continuous" dataType="double"/>\n')
    out.write('  <DataField name="species" optype="categorical" dataType="string">\n')
    for c in coefs:
        out.write(f'   <Value value="{c}"/>\n')
    out.write('  </DataField>\n </DataDictionary>\n')
    out.write(' <RegressionModel functionName="classification" normalizationMethod="softmax" modelName="iris_lr">\n')
    out.write('  <MiningSchema><MiningField name="species" usageType="target"/>')
    for f in fields:
        out.write(f'<MiningField name="{f}"/>')
    out.write('</MiningSchema>\n')
    out.write('  <Output>')
    for c in coefs:
        out.write(f'<OutputField name="probability({c})" optype="continuous" dataType="double" '
                  f'feature="probability" value="{c}"/>')
    out.write('</Output>\n')
    for c, (b, w) in coefs.items():
        out.write(f'  <RegressionTable intercept="{b}" targetCategory="{c}">')
        for f, x in zip(fields, w):
            out.write(f'<NumericPredictor name="{f}" coefficient="{x}"/>')
        out.write('</RegressionTable>\n')
    out.write(' </RegressionModel>\n</PMML>\n')
    return out.getvalue()


def mlp_pmml(n_features: int = 64, hidden: Tuple[int, ...] = (256, 256), n_out: int = 1, seed: int = 0,
             activation: str = "rectifier", classification: bool = False) -> str:
    """3-layer NeuralNetwork (``hidden`` layers + output layer), NormContinuous inputs."""
    rng = np.random.default_rng(seed)
    out = io.StringIO()
    _header(out, f"synthetic MLP {n_features}-{'-'.join(map(str, hidden))}-{n_out}")
    cats = [str(c) for c in range(n_out)] if classification else None
    _data_dictionary(out, n_features, "y", "integer" if classification else "double", cats)
    fn = "classification" if classification else "regression"
    out.write(f' <NeuralNetwork functionName="{fn}" activationFunction="{activation}">\n')
    _mining_schema(out, n_features, "y", "  ")
    out.write('  <NeuralInputs>\n')
    for j in range(n_features):
        mu, sd = rng.standard_normal() * 0.1, 1.0 + 0.1 * rng.random()
        out.write(f'   <NeuralInput id="i{j}"><DerivedField optype="continuous" dataType="double">'
                  f'<NormContinuous field="f{j}"><LinearNorm orig="{mu - sd:.6f}" norm="-1"/>'
                  f'<LinearNorm orig="{mu + sd:.6f}" norm="1"/></NormContinuous></DerivedField></NeuralInput>\n')
    out.write('  </NeuralInputs>\n')
    prev = [f"i{j}" for j in range(n_features)]
    dims = list(hidden) + [n_out]
    for li, width in enumerate(dims):
        last = li == len(dims) - 1
        attrs = ""
        if last:
            attrs = ' activationFunction="identity"' + (' normalizationMethod="softmax"' if classification else "")
        out.write(f'  <NeuralLayer{attrs}>\n')
        scale = 1.0 / np.sqrt(len(prev))
        W = rng.standard_normal((width, len(prev))) * scale
        b = rng.standard_normal(width) * 0.05
        ids = []
        for k in range(width):
            nid = f"n{li}_{k}"
            ids.append(nid)
            out.write(f'   <Neuron id="{nid}" bias="{b[k]:.7g}">')
            out.write("".join(f'<Con from="{p}" weight="{W[k, j]:.7g}"/>' for j, p in enumerate(prev)))
            out.write('</Neuron>\n')
        out.write('  </NeuralLayer>\n')
        prev = ids
    out.write('  <NeuralOutputs>\n')
    for k, nid in enumerate(prev):
        if classification:
            ex = f'<NormDiscrete field="y" value="{k}"/>'
        else:
            ex = '<FieldRef field="y"/>'
        out.write(f'   <NeuralOutput outputNeuron="{nid}"><DerivedField optype="continuous" dataType="double">'
                  f'{ex}</DerivedField></NeuralOutput>\n')
    out.write('  </NeuralOutputs>\n </NeuralNetwork>\n</PMML>\n')
    return out.getvalue()


def svm_pmml(n_features: int = 16, n_sv: int = 256, seed: int = 0, kernel: str = "radialBasis",
             classification: bool = True, gamma: float = 0.05, n_classes: int = 2) -> str:
    """libsvm / sklearn-style SVM PMML; ``n_classes > 2`` exports one-against-one machines (one per
    class pair, each over its own subset of the shared support vectors)."""
    rng = np.random.default_rng(seed)
    if classification and n_classes > 2:
        return _svm_ovo_pmml(rng, n_features, n_sv, kernel, gamma, n_classes)
    out = io.StringIO()
    _header(out, f"synthetic SVM {kernel} {n_sv} support vectors")
    cats = ["0", "1"] if classification else None
    _data_dictionary(out, n_features, "y", "integer" if classification else "double", cats)
    fn = "classification" if classification else "regression"
    out.write(f' <SupportVectorMachineModel functionName="{fn}" svmRepresentation="SupportVectors">\n')
    _mining_schema(out, n_features, "y", "  ")
    ktag = {"radialBasis": f'<RadialBasisKernelType gamma="{gamma}"/>', "linear": '<LinearKernelType/>',
            "polynomial": f'<PolynomialKernelType gamma="{gamma}" coef0="1" degree="3"/>',
            "sigmoid": f'<SigmoidKernelType gamma="{gamma}" coef0="0.5"/>'}[kernel]
    out.write(f'  {ktag}\n  <VectorDictionary numberOfVectors="{n_sv}">\n   <VectorFields numberOfFields="{n_features}">')
    out.write("".join(f'<FieldRef field="f{j}"/>' for j in range(n_features)))
    out.write('</VectorFields>\n')
    S = rng.standard_normal((n_sv, n_features))
    for i in range(n_sv):
        out.write(f'   <VectorInstance id="sv{i}"><Array n="{n_features}" type="real">'
                  + " ".join(f"{v:.6g}" for v in S[i]) + '</Array></VectorInstance>\n')
    out.write('  </VectorDictionary>\n')
    tc = ' targetCategory="0" alternateTargetCategory="1"' if classification else ""
    out.write(f'  <SupportVectorMachine{tc}>\n   <SupportVectors numberOfSupportVectors="{n_sv}">')
    out.write("".join(f'<SupportVector vectorId="sv{i}"/>' for i in range(n_sv)))
    out.write('</SupportVectors>\n')
    alpha = rng.standard_normal(n_sv) * 0.5
    out.write(f'   <Coefficients numberOfCoefficients="{n_sv}" absoluteValue="{rng.standard_normal() * 0.1:.6g}">')
    out.write("".join(f'<Coefficient value="{a:.6g}"/>' for a in alpha))
    out.write('</Coefficients>\n  </SupportVectorMachine>\n </SupportVectorMachineModel>\n</PMML>\n')
    return out.getvalue()


def kmeans_pmml(n_clusters: int = 64, n_features: int = 32, seed: int = 0, metric: str = "squaredEuclidean",
                weighted: bool = False, compare: str = "absDiff") -> str:
    """Centre-based ``ClusteringModel`` with ``n_clusters`` standard-normal centres (ids 1..K as the
    predicted value); ``weighted`` adds random ``ClusteringField`` field weights."""
    rng = np.random.default_rng(seed)
    out = io.StringIO()
    _header(out, f"synthetic k-means {n_clusters} clusters x {n_features} features")
    out.write(f' <DataDictionary numberOfFields="{n_features + 1}">\n')
    for j in range(n_features):
        out.write(f'  <DataField name="f{j}" optype="continuous" dataType="float"/>\n')
    out.write('  <DataField name="cluster" optype="categorical" dataType="string"/>\n </DataDictionary>\n')
    out.write(f' <ClusteringModel modelName="kmeans" functionName="clustering" modelClass="centerBased" '
              f'numberOfClusters="{n_clusters}">\n')
    out.write('  <MiningSchema>\n   <MiningField name="cluster" usageType="predicted"/>\n')
    for j in range(n_features):
        out.write(f'   <MiningField name="f{j}"/>\n')
    out.write('  </MiningSchema>\n')
    out.write(f'  <ComparisonMeasure kind="distance"><{metric}/></ComparisonMeasure>\n')
    for j in range(n_features):
        w = f' fieldWeight="{_fnum(rng.uniform(0.25, 2.0))}"' if weighted else ""
        out.write(f'  <ClusteringField field="f{j}" compareFunction="{compare}"{w}/>\n')
    C = rng.standard_normal((n_clusters, n_features))
    for k in range(n_clusters):
        out.write(f'  <Cluster id="{k + 1}" name="c{k + 1}"><Array n="{n_features}" type="real">'
                  + " ".join(_fnum(v) for v in C[k]) + '</Array></Cluster>\n')
    out.write(' </ClusteringModel>\n</PMML>\n')
    return out.getvalue()


_LEVELS = ("red", "green", "blue")


def _mixed_dictionary(out: io.StringIO, F: int, target: str, categories: Optional[List[str]]) -> None:
    out.write(f' <DataDictionary numberOfFields="{F + 2}">\n')
    for j in range(F):
        out.write(f'  <DataField name="f{j}" optype="continuous" dataType="double"/>\n')
    out.write('  <DataField name="color" optype="categorical" dataType="string">'
              + "".join(f'<Value value="{v}"/>' for v in _LEVELS) + '</DataField>\n')
    if categories is None:
        out.write(f'  <DataField name="{target}" optype="continuous" dataType="double"/>\n')
    else:
        out.write(f'  <DataField name="{target}" optype="categorical" dataType="string">'
                  + "".join(f'<Value value="{c}"/>' for c in categories) + '</DataField>\n')
    out.write(' </DataDictionary>\n')


def _mixed_schema(out: io.StringIO, F: int, target: str) -> None:
    out.write(f'  <MiningSchema>\n   <MiningField name="{target}" usageType="target"/>\n')
    for j in range(F):
        out.write(f'   <MiningField name="f{j}"/>\n')
    out.write('   <MiningField name="color"/>\n  </MiningSchema>\n')


def regression_design_pmml(n_features: int = 4, classes: int = 0, normalization: str = "none",
                           seed: int = 0) -> str:
    """``RegressionModel`` with exponents, a categorical predictor (string field ``color``) and
    interaction terms — the non-dense tables the design-matrix lowering handles. ``classes > 0``:
    one table per class."""
    rng = np.random.default_rng(seed)
    out = io.StringIO()
    _header(out, "synthetic regression with categorical predictors and terms")
    cats = [str(k) for k in range(classes)] if classes else None
    _mixed_dictionary(out, n_features, "y", cats)
    fn = "classification" if classes else "regression"
    out.write(f' <RegressionModel functionName="{fn}" normalizationMethod="{normalization}">\n')
    _mixed_schema(out, n_features, "y")
    for k in range(max(classes, 1)):
        tc = f' targetCategory="{k}"' if classes else ""
        out.write(f'  <RegressionTable intercept="{rng.normal():.6g}"{tc}>\n')
        for j in range(n_features):
            e = ' exponent="2"' if j % 3 == 1 else ""
            out.write(f'   <NumericPredictor name="f{j}"{e} coefficient="{rng.normal() * 0.5:.6g}"/>\n')
        for v in _LEVELS[:2]:
            out.write(f'   <CategoricalPredictor name="color" value="{v}" coefficient="{rng.normal():.6g}"/>\n')
        out.write(f'   <PredictorTerm coefficient="{rng.normal() * 0.3:.6g}"><FieldRef field="f0"/>'
                  f'<FieldRef field="f{n_features - 1}"/></PredictorTerm>\n')
        out.write('  </RegressionTable>\n')
    out.write(' </RegressionModel>\n</PMML>\n')
    return out.getvalue()


def glm_pmml(model_type: str = "generalizedLinear", link: str = "log", n_features: int = 3, seed: int = 0,
             classes: int = 3, binomial: Optional[str] = None, event_cells: bool = True) -> str:
    """``GeneralRegressionModel`` (PPMatrix / ParamMatrix) with covariates ``f*`` (one squared),
    factor ``color`` and a covariate x factor interaction. ``multinomialLogistic`` gets
    ``classes`` categories, the last one the reference; ``ordinalMultinomial`` gets ``classes``
    ordered categories, one increasing cut point (``p0``) per category but the last, the other
    parameters shared, and ``link`` as its ``cumulativeLink``. ``binomial`` ("first" / "last" /
    "default"): a classification ``generalizedLinear`` over categories "0" / "1" whose reference "0"
    is listed first, last, or left to the default (no attribute); ``event_cells`` puts the event's
    targetCategory on the PCells (else the cells carry none)."""
    rng = np.random.default_rng(seed)
    out = io.StringIO()
    _header(out, f"synthetic GLM {model_type} {link}")
    ordinal = model_type == "ordinalMultinomial"
    multi = model_type == "multinomialLogistic" or ordinal
    cats = [str(c) for c in range(classes)] if multi else None
    if binomial:
        cats = ["0", "1"] if binomial == "first" else ["1", "0"]  # reference "0" (numeric labels: Score values)
    _mixed_dictionary(out, n_features, "y", cats)
    fn = "classification" if multi or binomial else "regression"
    attrs = f' targetReferenceCategory="{classes - 1}"' if multi else f' linkFunction="{link}"'
    if ordinal:
        attrs = f' cumulativeLink="{link}"'
    if binomial in ("first", "last"):
        attrs += ' targetReferenceCategory="0"'
    if link == "power" and not multi:
        attrs += ' linkParameter="0"'
    out.write(f' <GeneralRegressionModel functionName="{fn}" modelType="{model_type}"{attrs} '
              f'offsetValue="0.25">\n')
    _mixed_schema(out, n_features, "y")
    params = ["p0"] + [f"p{j + 1}" for j in range(n_features)] + ["pc1", "pc2", "px"]
    out.write('  <ParameterList>' + "".join(f'<Parameter name="{p}"/>' for p in params) + '</ParameterList>\n')
    out.write('  <FactorList><Predictor name="color"/></FactorList>\n')
    out.write('  <CovariateList>' + "".join(f'<Predictor name="f{j}"/>' for j in range(n_features))
              + '</CovariateList>\n')
    out.write('  <PPMatrix>\n')
    for j in range(n_features):
        e = "2" if j == 1 else "1"
        out.write(f'   <PPCell value="{e}" predictorName="f{j}" parameterName="p{j + 1}"/>\n')
    out.write('   <PPCell value="red" predictorName="color" parameterName="pc1"/>\n')
    out.write('   <PPCell value="green" predictorName="color" parameterName="pc2"/>\n')
    out.write('   <PPCell value="blue" predictorName="color" parameterName="px"/>\n')
    out.write('   <PPCell value="1" predictorName="f0" parameterName="px"/>\n')
    out.write('  </PPMatrix>\n  <ParamMatrix>\n')
    if ordinal:
        cuts = np.sort(rng.normal(size=classes - 1)) * 1.5
        for c, cut in zip(cats[:-1], cuts):
            out.write(f'   <PCell parameterName="p0" targetCategory="{c}" beta="{cut:.6g}"/>\n')
        for p in params[1:]:
            out.write(f'   <PCell parameterName="{p}" beta="{rng.normal() * 0.5:.6g}"/>\n')
    for c in ([] if ordinal else cats[:-1] if multi else ["1" if event_cells else None] if binomial else [None]):
        tc = f' targetCategory="{c}"' if c is not None else ""
        for p in params:
            out.write(f'   <PCell parameterName="{p}"{tc} beta="{rng.normal() * 0.3:.6g}"/>\n')
    out.write('  </ParamMatrix>\n </GeneralRegressionModel>\n</PMML>\n')
    return out.getvalue()


def scorecard_pmml(n_features: int = 4, seed: int = 0, reason_codes: bool = True, missing_attribute: bool = True) -> str:
    """``Scorecard`` over ``f*`` (3 interval bins each, the middle one a compound ``and``) and the
    categorical ``color`` (set + equality attributes); with ``missing_attribute`` the first
    characteristic also matches missing values (``isMissing``)."""
    rng = np.random.default_rng(seed)
    out = io.StringIO()
    _header(out, "synthetic scorecard")
    _mixed_dictionary(out, n_features, "score", None)
    rc = ' useReasonCodes="true" reasonCodeAlgorithm="pointsBelow" baselineScore="10"' if reason_codes \
        else ' useReasonCodes="false"'
    out.write(f' <Scorecard functionName="regression" initialScore="{rng.uniform(-5, 5):.4f}"{rc}>\n')
    _mixed_schema(out, n_features, "score")
    if reason_codes:
        out.write('  <Output>\n   <OutputField name="RC1" feature="reasonCode" rank="1" dataType="string"/>\n'
                  '   <OutputField name="RC2" feature="reasonCode" rank="2" dataType="string"/>\n  </Output>\n')
    out.write('  <Characteristics>\n')
    for j in range(n_features):
        a, b = sorted(rng.normal(size=2))
        out.write(f'   <Characteristic name="ch{j}" reasonCode="R{j}">\n')
        if missing_attribute and j == 0:
            out.write(f'    <Attribute partialScore="{rng.uniform(0, 20):.3f}"><SimplePredicate field="f{j}" '
                      'operator="isMissing"/></Attribute>\n')
        out.write(f'    <Attribute partialScore="{rng.uniform(0, 20):.3f}"><SimplePredicate field="f{j}" '
                  f'operator="lessThan" value="{a:.4f}"/></Attribute>\n')
        out.write(f'    <Attribute partialScore="{rng.uniform(0, 20):.3f}" reasonCode="R{j}m"><CompoundPredicate '
                  f'booleanOperator="and"><SimplePredicate field="f{j}" operator="greaterOrEqual" value="{a:.4f}"/>'
                  f'<SimplePredicate field="f{j}" operator="lessThan" value="{b:.4f}"/></CompoundPredicate>'
                  '</Attribute>\n')
        out.write(f'    <Attribute partialScore="{rng.uniform(0, 20):.3f}"><SimplePredicate field="f{j}" '
                  f'operator="greaterOrEqual" value="{b:.4f}"/></Attribute>\n')
        out.write('   </Characteristic>\n')
    out.write('   <Characteristic name="color" reasonCode="RC" baselineScore="5">\n')
    out.write(f'    <Attribute partialScore="{rng.uniform(0, 20):.3f}"><SimpleSetPredicate field="color" '
              'booleanOperator="isIn"><Array n="2" type="string">red green</Array></SimpleSetPredicate></Attribute>\n')
    out.write(f'    <Attribute partialScore="{rng.uniform(0, 20):.3f}"><SimplePredicate field="color" '
              'operator="equal" value="blue"/></Attribute>\n')
    out.write(f'    <Attribute partialScore="{rng.uniform(0, 20):.3f}"><True/></Attribute>\n')
    out.write('   </Characteristic>\n  </Characteristics>\n </Scorecard>\n</PMML>\n')
    return out.getvalue()


def ruleset_pmml(n_features: int = 4, n_rules: int = 12, criterion: str = "firstHit", seed: int = 0,
                 default: bool = True, classes: int = 3) -> str:
    """``RuleSetModel`` with simple rules on ``f*`` / ``color`` and one ``CompoundRule``."""
    rng = np.random.default_rng(seed)
    out = io.StringIO()
    _header(out, f"synthetic rule set {criterion}")
    cats = [str(k) for k in range(classes)]
    _mixed_dictionary(out, n_features, "y", cats)
    out.write(' <RuleSetModel functionName="classification">\n')
    _mixed_schema(out, n_features, "y")
    dflt = ' defaultScore="0" defaultConfidence="0.5"' if default else ""
    out.write(f'  <RuleSet{dflt}>\n   <RuleSelectionMethod criterion="{criterion}"/>\n')

    def pred() -> str:
        j = int(rng.integers(n_features))
        op = ["lessThan", "greaterOrEqual", "greaterThan"][int(rng.integers(3))]
        p = f'<SimplePredicate field="f{j}" operator="{op}" value="{rng.normal():.4f}"/>'
        if rng.random() < 0.3:
            p = (f'<CompoundPredicate booleanOperator="and">{p}<SimplePredicate field="color" operator="notEqual" '
                 f'value="{_LEVELS[int(rng.integers(3))]}"/></CompoundPredicate>')
        return p

    def rule(i: int) -> str:
        return (f'   <SimpleRule id="r{i}" score="{cats[int(rng.integers(classes))]}" weight="{rng.uniform(0.1, 2):.3f}" '
                f'confidence="{rng.uniform(0.5, 1):.3f}">{pred()}</SimpleRule>\n')

    for i in range(n_rules // 2):
        out.write(rule(i))
    out.write(f'   <CompoundRule>{pred()}\n')
    for i in range(n_rules // 2, n_rules - 2):
        out.write(rule(i))
    out.write('   </CompoundRule>\n')
    for i in range(n_rules - 2, n_rules):
        out.write(rule(i))
    out.write('  </RuleSet>\n </RuleSetModel>\n</PMML>\n')
    return out.getvalue()


def naive_bayes_pmml(n_features: int = 4, classes: int = 3, seed: int = 0, threshold: float = 0.001,
                     discretized: Optional[str] = None) -> str:
    """``NaiveBayesModel``: Gaussian ``f*`` inputs and the categorical ``color`` (one level never
    seen with class 0: exercises the threshold). ``discretized``: the last ``f`` input becomes
    three Discretize bins with PairCounts — ``"inline"`` as the BayesInput's own DerivedField,
    ``"local"`` as a LocalTransformations field ``fbin`` the BayesInput names."""
    rng = np.random.default_rng(seed)
    out = io.StringIO()
    _header(out, "synthetic naive Bayes")
    cats = [str(k) for k in range(classes)]
    _mixed_dictionary(out, n_features, "y", cats)
    out.write(f' <NaiveBayesModel functionName="classification" threshold="{threshold}">\n')
    _mixed_schema(out, n_features, "y")
    last = n_features - 1
    disc = (f'<Discretize field="f{last}"><DiscretizeBin binValue="low"><Interval closure="openOpen" '
            'rightMargin="-0.5"/></DiscretizeBin><DiscretizeBin binValue="mid"><Interval closure="closedOpen" '
            'leftMargin="-0.5" rightMargin="0.5"/></DiscretizeBin><DiscretizeBin binValue="high"><Interval '
            'closure="closedOpen" leftMargin="0.5"/></DiscretizeBin></Discretize>')
    if discretized == "local":
        out.write(f'  <LocalTransformations><DerivedField name="fbin" optype="categorical" dataType="string">'
                  f'{disc}</DerivedField></LocalTransformations>\n')
    counts = rng.integers(50, 200, classes)
    out.write('  <BayesInputs>\n')
    for j in range(n_features):
        if discretized and j == last:
            name = "fbin" if discretized == "local" else f"f{j}"
            inner = ("" if discretized == "local"
                     else f'<DerivedField optype="categorical" dataType="string">{disc}</DerivedField>')
            out.write(f'   <BayesInput fieldName="{name}">{inner}')
            for b in ("low", "mid", "high"):
                out.write(f'<PairCounts value="{b}"><TargetValueCounts>'
                          + "".join(f'<TargetValueCount value="{cats[k]}" count="{int(rng.integers(5, 60))}"/>'
                                    for k in range(classes)) + '</TargetValueCounts></PairCounts>')
            out.write('</BayesInput>\n')
            continue
        out.write(f'   <BayesInput fieldName="f{j}"><TargetValueStats>')
        for k in range(classes):
            out.write(f'<TargetValueStat value="{cats[k]}"><GaussianDistribution mean="{rng.normal() * 0.7:.4f}" '
                      f'variance="{rng.uniform(0.5, 2.0):.4f}"/></TargetValueStat>')
        out.write('</TargetValueStats></BayesInput>\n')
    out.write('   <BayesInput fieldName="color">\n')
    for li, lvl in enumerate(_LEVELS):
        out.write(f'    <PairCounts value="{lvl}"><TargetValueCounts>')
        for k in range(classes):
            cnt = 0 if (li == 2 and k == 0) else int(rng.integers(5, counts[k] // 3))
            out.write(f'<TargetValueCount value="{cats[k]}" count="{cnt}"/>')
        out.write('</TargetValueCounts></PairCounts>\n')
    out.write('   </BayesInput>\n  </BayesInputs>\n')
    out.write('  <BayesOutput fieldName="y"><TargetValueCounts>'
              + "".join(f'<TargetValueCount value="{cats[k]}" count="{counts[k]}"/>' for k in range(classes))
              + '</TargetValueCounts></BayesOutput>\n')
    out.write(' </NaiveBayesModel>\n</PMML>\n')
    return out.getvalue()


def knn_pmml(n_instances: int = 200, n_features: int = 4, k: int = 3, classification: bool = True, seed: int = 0,
             method: Optional[str] = None, metric: str = "euclidean", classes: int = 3,
             measure: str = "distance", compare: Optional[str] = None, target: Optional[str] = None,
             threshold: float = 0.001, quantum: Optional[float] = None) -> str:
    """``NearestNeighborModel`` over ``n_instances`` inline training rows of ``f*`` (targets
    ``0..classes-1`` or real values). ``metric`` is the ComparisonMeasure element body (e.g.
    ``'minkowski p-parameter="3"'``), ``measure`` its kind, ``compare`` a compareFunction, ``target``
    the attributes of a ``<Target field="y" .../>`` (regression rescale / clip / cast), ``threshold``
    the weighting offset, ``quantum`` rounds the instances to multiples of it (exact in fp32)."""
    rng = np.random.default_rng(seed)
    out = io.StringIO()
    _header(out, f"synthetic {k}-NN")
    cats = [str(c) for c in range(classes)] if classification else None
    _data_dictionary(out, n_features, "y", "string" if classification else "double", cats)
    fn = "classification" if classification else "regression"
    meth = (f' categoricalScoringMethod="{method or "majorityVote"}"' if classification
            else f' continuousScoringMethod="{method or "average"}"')
    out.write(f' <NearestNeighborModel functionName="{fn}" numberOfNeighbors="{k}"{meth} threshold="{threshold!r}">\n')
    _mining_schema(out, n_features, "y", "  ")
    if target:
        out.write(f'  <Targets><Target field="y" {target}/></Targets>\n')
    out.write(f'  <TrainingInstances recordCount="{n_instances}" fieldCount="{n_features + 1}">\n   <InstanceFields>')
    out.write("".join(f'<InstanceField field="f{j}" column="c{j}"/>' for j in range(n_features)))
    out.write('<InstanceField field="y" column="target"/></InstanceFields>\n   <InlineTable>\n')
    X = rng.standard_normal((n_instances, n_features))
    if quantum:
        X = np.round(X / quantum) * quantum
    for i in range(n_instances):
        t = str(int(rng.integers(classes))) if classification else f"{rng.normal() * 3:.4f}"
        out.write("    <row>" + "".join(f"<c{j}>{X[i, j]:.5f}</c{j}>" for j in range(n_features))
                  + f"<target>{t}</target></row>\n")
    out.write('   </InlineTable>\n  </TrainingInstances>\n')
    cf = f' compareFunction="{compare}"' if compare else ""
    out.write(f'  <ComparisonMeasure kind="{measure}"{cf}><{metric}/></ComparisonMeasure>\n  <KNNInputs>')
    out.write("".join(f'<KNNInput field="f{j}"/>' for j in range(n_features)))
    out.write('</KNNInputs>\n </NearestNeighborModel>\n</PMML>\n')
    return out.getvalue()


def mixed_records(n_rows: int, n_features: int, seed: int = 0, missing_rate: float = 0.0) -> Tuple[list, np.ndarray]:
    """Records for the ``_mixed_dictionary`` models: ``(list of dicts, [rows, F+1] float matrix with
    the color vocabulary code in the last column)``."""
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n_rows, n_features + 1))
    X[:, -1] = rng.integers(0, len(_LEVELS), n_rows)
    if missing_rate > 0:
        X[rng.random(X.shape) < missing_rate] = np.nan
    recs = []
    for r in X:
        d = {f"f{j}": float(r[j]) for j in range(n_features) if not np.isnan(r[j])}
        if not np.isnan(r[-1]):
            d["color"] = _LEVELS[int(r[-1])]
        recs.append(d)
    return recs, X


def stream_matrix(n_rows: int, n_features: int, seed: int = 0, missing_rate: float = 0.0) -> np.ndarray:
    """Synthetic fp32 record batch ``[rows, features]`` (standard normal; NaN = missing)."""
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n_rows, n_features), dtype=np.float32)
    if missing_rate > 0:
        X[rng.random((n_rows, n_features)) < missing_rate] = np.nan
    return X


def set_target(txt: str, field: str = "y", min: Optional[float] = None, max: Optional[float] = None,
               factor: float = 1.0, constant: float = 0.0, cast: Optional[str] = None,
               default: Optional[float] = None) -> str:
    """Replace (or insert) the top-level model's ``<Targets>`` with one ``Target`` carrying the
    given min / max / rescale / castInteger / TargetValue defaultValue."""
    import re

    attrs = f'field="{field}" rescaleFactor="{_fnum(factor)}" rescaleConstant="{_fnum(constant)}"'
    if min is not None:
        attrs += f' min="{_fnum(min)}"'
    if max is not None:
        attrs += f' max="{_fnum(max)}"'
    if cast is not None:
        attrs += f' castInteger="{cast}"'
    body = f'<TargetValue defaultValue="{_fnum(default)}"/>' if default is not None else ""
    new = f'<Targets><Target {attrs}>{body}</Target></Targets>'
    m = re.search(r"<Targets>.*?</Targets>", txt, flags=re.S)
    if m is not None and m.start() < txt.find("<Segment"):
        return txt[:m.start()] + new + txt[m.end():]
    i = txt.find("</MiningSchema>") + len("</MiningSchema>")
    return txt[:i] + "\n  " + new + txt[i:]


def segmented_pmml(method: str = "selectFirst", classification: bool = False, n_segments: int = 4,
                   depth: int = 3, n_features: int = 6, n_classes: int = 3, seed: int = 0,
                   predicates: bool = True, missing_treatment: Optional[str] = None,
                   linear_segment: bool = False) -> str:
    """MiningModel with per-segment predicates over small trees (and optionally one
    RegressionModel segment): ``selectFirst`` / ``max`` / ``min`` / ``median`` / ``sum`` /
    ``average`` / ``weightedAverage`` (regression) or ``majorityVote`` / ``weightedMajorityVote``
    / ``selectFirst`` (classification) — the segmentations the fused ensemble kernels refuse.
    Segment predicates mix Simple (incl. isMissing), SimpleSet and Compound(and/or/surrogate)."""
    rng = np.random.default_rng(seed)
    thresholds = np.sort(rng.standard_normal((n_features, 64)).astype(np.float32), axis=1)
    cats = [str(c) for c in range(n_classes)]
    out = io.StringIO()
    _header(out, f"synthetic segmented MiningModel ({method})")
    _data_dictionary(out, n_features, "y", "integer" if classification else "double",
                     cats if classification else None)
    fn = "classification" if classification else "regression"
    mpt = f' missingPredictionTreatment="{missing_treatment}"' if missing_treatment else ""
    out.write(f' <MiningModel functionName="{fn}">\n')
    _mining_schema(out, n_features, "y", "  ")
    out.write(f'  <Segmentation multipleModelMethod="{method}"{mpt}>\n')

    def pred(i: int) -> str:
        if not predicates:
            return "<True/>"
        f, g = int(rng.integers(n_features)), int(rng.integers(n_features))
        v = _fnum(float(rng.standard_normal() * 0.5))
        kind = i % 5
        if kind == 0:
            return f'<SimplePredicate field="f{f}" operator="greaterThan" value="{v}"/>'
        if kind == 1:
            return (f'<CompoundPredicate booleanOperator="and"><SimplePredicate field="f{f}" operator="lessOrEqual" '
                    f'value="{v}"/><SimplePredicate field="f{g}" operator="notEqual" value="0"/></CompoundPredicate>')
        if kind == 2:
            return (f'<CompoundPredicate booleanOperator="surrogate"><SimplePredicate field="f{f}" '
                    f'operator="lessThan" value="{v}"/><SimplePredicate field="f{g}" operator="isMissing"/>'
                    '</CompoundPredicate>')
        if kind == 3:
            return (f'<CompoundPredicate booleanOperator="or"><SimplePredicate field="f{f}" operator="greaterOrEqual" '
                    f'value="{v}"/><SimplePredicate field="f{g}" operator="isMissing"/></CompoundPredicate>')
        return "<True/>"

    for i in range(n_segments):
        w = _fnum(float(rng.uniform(0.5, 2.0)))
        out.write(f'   <Segment id="{i + 1}" weight="{w}">{pred(i)}\n')
        if linear_segment and i == n_segments - 1 and not classification:
            out.write('    <RegressionModel functionName="regression">\n')
            _mining_schema(out, n_features, "y", "     ")
            out.write(f'     <RegressionTable intercept="{_fnum(float(rng.standard_normal()))}">')
            for j in range(n_features):
                out.write(f'<NumericPredictor name="f{j}" coefficient="{_fnum(float(rng.standard_normal()))}"/>')
            out.write('</RegressionTable>\n    </RegressionModel>\n')
        else:
            g = _TreeGen(rng, n_features, depth, 0.9, thresholds)
            out.write(f'    <TreeModel functionName="{fn}" missingValueStrategy="defaultChild" '
                      'splitCharacteristic="binarySplit">\n')
            _mining_schema(out, n_features, "y", "     ")
            leaf = (lambda: cats[int(rng.integers(n_classes))]) if classification \
                else (lambda: _fnum(float(rng.standard_normal())))
            g.write(out, 0, "<True/>", leaf, "     ", force_split=True)
            out.write('    </TreeModel>\n')
        out.write('   </Segment>\n')
    out.write('  </Segmentation>\n </MiningModel>\n</PMML>\n')
    return out.getvalue()


def _svm_ovo_pmml(rng, n_features: int, n_sv: int, kernel: str, gamma: float, n_classes: int) -> str:
    out = io.StringIO()
    _header(out, f"synthetic one-against-one SVM {kernel} {n_classes} classes")
    cats = [str(c) for c in range(n_classes)]
    _data_dictionary(out, n_features, "y", "integer", cats)
    out.write(' <SupportVectorMachineModel functionName="classification" svmRepresentation="SupportVectors" '
              'classificationMethod="OneAgainstOne">\n')
    _mining_schema(out, n_features, "y", "  ")
    ktag = {"radialBasis": f'<RadialBasisKernelType gamma="{gamma}"/>', "linear": '<LinearKernelType/>',
            "polynomial": f'<PolynomialKernelType gamma="{gamma}" coef0="1" degree="3"/>',
            "sigmoid": f'<SigmoidKernelType gamma="{gamma}" coef0="0.5"/>'}[kernel]
    out.write(f'  {ktag}\n  <VectorDictionary numberOfVectors="{n_sv}">\n   <VectorFields numberOfFields="{n_features}">')
    out.write("".join(f'<FieldRef field="f{j}"/>' for j in range(n_features)))
    out.write('</VectorFields>\n')
    S = rng.standard_normal((n_sv, n_features))
    for i in range(n_sv):
        out.write(f'   <VectorInstance id="sv{i}"><Array n="{n_features}" type="real">'
                  + " ".join(f"{v:.6g}" for v in S[i]) + '</Array></VectorInstance>\n')
    out.write('  </VectorDictionary>\n')
    owner = rng.integers(n_classes, size=n_sv)  # each support vector belongs to one class
    for a in range(n_classes):
        for b in range(a + 1, n_classes):
            ids = [i for i in range(n_sv) if owner[i] in (a, b)]
            out.write(f'  <SupportVectorMachine targetCategory="{cats[a]}" alternateTargetCategory="{cats[b]}">\n'
                      f'   <SupportVectors numberOfSupportVectors="{len(ids)}">')
            out.write("".join(f'<SupportVector vectorId="sv{i}"/>' for i in ids))
            out.write('</SupportVectors>\n')
            coef = rng.standard_normal(len(ids)) * 0.5
            out.write(f'   <Coefficients numberOfCoefficients="{len(ids)}" '
                      f'absoluteValue="{rng.standard_normal() * 0.1:.6g}">')
            out.write("".join(f'<Coefficient value="{c:.6g}"/>' for c in coef))
            out.write('</Coefficients>\n  </SupportVectorMachine>\n')
    out.write(' </SupportVectorMachineModel>\n</PMML>\n')
    return out.getvalue()
