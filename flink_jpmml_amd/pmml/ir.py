"""Typed intermediate representation of a PMML document (PMML 3.0 - 4.4).

The parser (`parser.py`) builds these plain dataclasses from XML; the model families in
``flink_jpmml_amd.models`` evaluate them (float64 oracle) and compile them to device layouts.

This replaces what the reference obtains from ``JAXBUtil.unmarshalPMML`` +
``ModelEvaluatorFactory.newModelEvaluator`` (`S/api/PmmlModel.scala:53-61`).
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple

# --------------------------------------------------------------------------- dictionary


@dataclass
class Interval:
    closure: str  # openClosed | openOpen | closedOpen | closedClosed
    left: Optional[float]
    right: Optional[float]

    def contains(self, v: float) -> bool:
        lo_ok = True
        hi_ok = True
        if self.left is not None:
            lo_ok = v >= self.left if self.closure.startswith("closed") else v > self.left
        if self.right is not None:
            hi_ok = v <= self.right if self.closure.endswith("Closed") else v < self.right
        return lo_ok and hi_ok


@dataclass
class DataField:
    name: str
    optype: str  # continuous | categorical | ordinal
    data_type: str  # string | integer | float | double | boolean | date...
    values: List[str] = field(default_factory=list)  # property="valid" (default)
    invalid_values: List[str] = field(default_factory=list)
    missing_values: List[str] = field(default_factory=list)
    intervals: List[Interval] = field(default_factory=list)
    display_name: Optional[str] = None

    @property
    def is_string(self) -> bool:
        return self.data_type == "string"


@dataclass
class MiningField:
    name: str
    usage_type: str = "active"
    optype: Optional[str] = None
    invalid_value_treatment: str = "returnInvalid"  # returnInvalid | asIs | asMissing | asValue
    invalid_value_replacement: Optional[str] = None
    missing_value_replacement: Optional[str] = None
    missing_value_treatment: Optional[str] = None
    outliers: str = "asIs"  # asIs | asMissingValues | asExtremeValues
    low_value: Optional[float] = None
    high_value: Optional[float] = None
    importance: Optional[float] = None


@dataclass
class MiningSchema:
    fields: List[MiningField] = field(default_factory=list)

    def by_usage(self, *usages: str) -> List[MiningField]:
        return [f for f in self.fields if f.usage_type in usages]

    @property
    def active(self) -> List[MiningField]:
        return self.by_usage("active")

    @property
    def targets(self) -> List[MiningField]:
        return self.by_usage("predicted", "target")

    def get(self, name: str) -> Optional[MiningField]:
        for f in self.fields:
            if f.name == name:
                return f
        return None


# --------------------------------------------------------------------------- expressions


@dataclass
class Expression:
    pass


@dataclass
class Constant(Expression):
    value: Optional[str]
    data_type: Optional[str] = None
    missing: bool = False


@dataclass
class FieldRef(Expression):
    field: str
    map_missing_to: Optional[str] = None


@dataclass
class LinearNorm:
    orig: float
    norm: float


@dataclass
class NormContinuous(Expression):
    field: str
    norms: List[LinearNorm]
    outliers: str = "asIs"  # asIs | asMissingValues | asExtremeValues
    map_missing_to: Optional[float] = None


@dataclass
class NormDiscrete(Expression):
    field: str
    value: str
    map_missing_to: Optional[float] = None


@dataclass
class DiscretizeBin:
    bin_value: str
    interval: Interval


@dataclass
class Discretize(Expression):
    field: str
    bins: List[DiscretizeBin]
    map_missing_to: Optional[str] = None
    default_value: Optional[str] = None
    data_type: Optional[str] = None


@dataclass
class MapValues(Expression):
    output_column: str
    field_columns: List[Tuple[str, str]]  # (field name, column name)
    rows: List[Dict[str, str]]
    map_missing_to: Optional[str] = None
    default_value: Optional[str] = None
    data_type: Optional[str] = None


@dataclass
class Apply(Expression):
    function: str
    args: List[Expression]
    map_missing_to: Optional[str] = None
    default_value: Optional[str] = None
    invalid_value_treatment: str = "returnInvalid"


@dataclass
class DerivedField:
    name: str
    optype: Optional[str]
    data_type: Optional[str]
    expression: Expression
    values: List[str] = field(default_factory=list)


# --------------------------------------------------------------------------- predicates


@dataclass
class Predicate:
    pass


@dataclass
class TruePredicate(Predicate):
    pass


@dataclass
class FalsePredicate(Predicate):
    pass


@dataclass
class SimplePredicate(Predicate):
    field: str
    operator: str  # equal notEqual lessThan lessOrEqual greaterThan greaterOrEqual isMissing isNotMissing
    value: Optional[str] = None


@dataclass
class SimpleSetPredicate(Predicate):
    field: str
    boolean_operator: str  # isIn | isNotIn
    values: List[str] = field(default_factory=list)


@dataclass
class CompoundPredicate(Predicate):
    boolean_operator: str  # and | or | xor | surrogate
    predicates: List[Predicate] = field(default_factory=list)


# --------------------------------------------------------------------------- output / targets


@dataclass
class OutputField:
    name: str
    optype: Optional[str] = None
    data_type: Optional[str] = None
    target_field: Optional[str] = None
    feature: str = "predictedValue"
    value: Optional[str] = None
    segment_id: Optional[str] = None
    rank: int = 1
    is_final_result: bool = True
    expression: Optional[Expression] = None
    # association rules (feature="ruleValue" / "entityId" on an AssociationModel)
    rule_feature: str = "consequent"
    algorithm: str = "exclusiveRecommendation"
    rank_basis: str = "confidence"
    rank_order: str = "descending"


@dataclass
class TargetValue:
    value: Optional[str] = None
    display_value: Optional[str] = None
    prior_probability: Optional[float] = None
    default_value: Optional[float] = None


@dataclass
class Target:
    field: Optional[str]
    optype: Optional[str] = None
    cast_integer: Optional[str] = None  # round | ceiling | floor
    min: Optional[float] = None
    max: Optional[float] = None
    rescale_factor: float = 1.0
    rescale_constant: float = 0.0
    values: List[TargetValue] = field(default_factory=list)


# --------------------------------------------------------------------------- models


@dataclass
class Model:
    """Common part of every PMML model element."""

    element: str
    model_name: Optional[str]
    function_name: str
    mining_schema: MiningSchema
    output: List[OutputField] = field(default_factory=list)
    targets: List[Target] = field(default_factory=list)
    local_transformations: List[DerivedField] = field(default_factory=list)
    is_scorable: bool = True
    algorithm_name: Optional[str] = None
    math_context: Optional[str] = None  # x-mathContext: "float" | "double" (pmml/mathcontext.py)


# clustering ---------------------------------------------------------------


@dataclass
class ClusteringField:
    field: str
    weight: float = 1.0
    compare_function: Optional[str] = None
    similarity_scale: Optional[float] = None
    is_center_field: bool = True


@dataclass
class Cluster:
    name: Optional[str]
    id: Optional[str]
    center: List[float]
    size: Optional[int] = None


@dataclass
class ClusteringModel(Model):
    model_class: str = "centerBased"
    measure_kind: str = "distance"  # distance | similarity
    metric: str = "squaredEuclidean"
    minkowski_p: float = 2.0
    compare_function: str = "absDiff"
    fields: List[ClusteringField] = field(default_factory=list)
    clusters: List[Cluster] = field(default_factory=list)
    missing_value_weights: Optional[List[float]] = None


# trees ----------------------------------------------------------------------


@dataclass
class ScoreDistribution:
    value: str
    record_count: float
    probability: Optional[float] = None
    confidence: Optional[float] = None


@dataclass
class Node:
    id: Optional[str]
    score: Optional[str]
    predicate: Predicate
    children: List["Node"] = field(default_factory=list)
    record_count: Optional[float] = None
    default_child: Optional[str] = None
    distributions: List[ScoreDistribution] = field(default_factory=list)
    value_field: Optional[str] = None  # leaf score read per record from this field (complex scorecards)


@dataclass
class TreeModel(Model):
    root: Node = None  # type: ignore[assignment]
    missing_value_strategy: str = "none"
    missing_value_penalty: float = 1.0
    no_true_child_strategy: str = "returnNullPrediction"
    split_characteristic: str = "multiSplit"
    flat: Any = field(default=None, repr=False, compare=False)
    """:class:`~flink_jpmml_amd.pmml.flat.FlatTree` when the body came from the streaming scanner
    (``root`` is then materialised from it on first access)."""


def _tree_root_get(self):
    r = self.__dict__.get("_root")
    if r is None:
        flat = self.__dict__.get("flat")
        if flat is not None:
            r = self.__dict__["_root"] = flat.materialize()
    return r


def _tree_root_set(self, v):
    self.__dict__["_root"] = v


TreeModel.root = property(_tree_root_get, _tree_root_set)  # type: ignore[assignment]


# mining ---------------------------------------------------------------------


@dataclass
class Segment:
    id: Optional[str]
    weight: float
    predicate: Predicate
    model: Model


@dataclass
class MiningModel(Model):
    multiple_model_method: str = "sum"
    segments: List[Segment] = field(default_factory=list)
    missing_prediction_treatment: str = "continue"
    missing_threshold: float = 1.0


# regression -----------------------------------------------------------------


@dataclass
class NumericPredictor:
    name: str
    coefficient: float
    exponent: float = 1.0


@dataclass
class CategoricalPredictor:
    name: str
    value: str
    coefficient: float


@dataclass
class PredictorTerm:
    fields: List[str]
    coefficient: float


@dataclass
class RegressionTable:
    intercept: float
    target_category: Optional[str] = None
    numeric: List[NumericPredictor] = field(default_factory=list)
    categorical: List[CategoricalPredictor] = field(default_factory=list)
    terms: List[PredictorTerm] = field(default_factory=list)


@dataclass
class RegressionModel(Model):
    normalization_method: str = "none"
    tables: List[RegressionTable] = field(default_factory=list)


@dataclass
class GeneralRegressionModel(Model):
    """GLM subset: ``generalizedLinear``/``regression``/``multinomialLogistic`` with PPMatrix
    and ParamMatrix; lowered to :class:`RegressionModel` semantics by the evaluator."""

    model_type: str = "regression"
    link_function: Optional[str] = None
    link_power: Optional[float] = None
    distribution: Optional[str] = None
    offset_value: float = 0.0
    parameters: List[str] = field(default_factory=list)
    factors: List[str] = field(default_factory=list)
    covariates: List[str] = field(default_factory=list)
    pp_cells: List[Tuple[str, str, str]] = field(default_factory=list)  # (predictor, parameter, value)
    p_cells: List[Tuple[str, Optional[str], float]] = field(default_factory=list)  # (parameter, targetCategory, beta)
    target_reference_category: Optional[str] = None
    cumulative_link: Optional[str] = None  # ordinalMultinomial: logit | probit | cloglog | loglog | cauchit


# neural network --------------------------------------------------------------


@dataclass
class Neuron:
    id: str
    bias: float = 0.0
    width: Optional[float] = None
    altitude: Optional[float] = None
    connections: List[Tuple[str, float]] = field(default_factory=list)


@dataclass
class NeuralLayer:
    neurons: List[Neuron]
    activation: Optional[str] = None
    threshold: Optional[float] = None
    width: Optional[float] = None
    altitude: Optional[float] = None
    normalization: Optional[str] = None


@dataclass
class NeuralInput:
    id: str
    derived: DerivedField


@dataclass
class NeuralOutput:
    neuron: str
    derived: DerivedField


@dataclass
class NeuralNetwork(Model):
    activation: str = "logistic"
    normalization: str = "none"
    threshold: float = 0.0
    width: Optional[float] = None
    altitude: float = 1.0
    inputs: List[NeuralInput] = field(default_factory=list)
    layers: List[NeuralLayer] = field(default_factory=list)
    outputs: List[NeuralOutput] = field(default_factory=list)


# support vector machine ------------------------------------------------------


@dataclass
class SvmKernel:
    kind: str  # linear | polynomial | radialBasis | sigmoid
    gamma: float = 1.0
    coef0: float = 1.0
    degree: float = 1.0


@dataclass
class SupportVectorMachine:
    target_category: Optional[str]
    alternate_target_category: Optional[str]
    threshold: Optional[float]
    vector_ids: List[str]
    coefficients: List[float]
    intercept: float


@dataclass
class SupportVectorMachineModel(Model):
    kernel: SvmKernel = None  # type: ignore[assignment]
    representation: str = "SupportVectors"
    classification_method: str = "OneAgainstAll"
    threshold: float = 0.0
    max_wins: bool = False
    vector_fields: List[str] = field(default_factory=list)
    vectors: Dict[str, List[float]] = field(default_factory=dict)
    machines: List[SupportVectorMachine] = field(default_factory=list)


# --------------------------------------------------------------------------- document


@dataclass
class PMMLDocument:
    version: str
    data_fields: Dict[str, DataField]
    transformations: List[DerivedField]
    models: List[Model]
    header: Dict[str, Any] = field(default_factory=dict)

    @property
    def model(self) -> Model:
        """First scorable model (JPMML's ``ModelEvaluatorFactory`` picks the first one too)."""
        for m in self.models:
            if m.is_scorable:
                return m
        raise IndexError("PMML document contains no scorable model")


# scorecard / rule set -------------------------------------------------------


@dataclass
class ScorecardAttribute:
    predicate: Predicate
    partial_score: Optional[float]
    reason_code: Optional[str] = None
    complex_score: Optional["Expression"] = None  # ComplexPartialScore: evaluated per record


@dataclass
class Characteristic:
    name: Optional[str]
    attributes: List[ScorecardAttribute] = field(default_factory=list)
    reason_code: Optional[str] = None
    baseline_score: Optional[float] = None


@dataclass
class Scorecard(Model):
    initial_score: float = 0.0
    use_reason_codes: bool = True
    reason_code_algorithm: str = "pointsBelow"
    baseline_score: Optional[float] = None
    baseline_method: str = "other"
    characteristics: List[Characteristic] = field(default_factory=list)


@dataclass
class SimpleRule:
    id: Optional[str]
    score: str
    predicate: Predicate
    confidence: float = 1.0
    weight: float = 1.0
    distributions: List[ScoreDistribution] = field(default_factory=list)


@dataclass
class CompoundRule:
    predicate: Predicate
    rules: List[object] = field(default_factory=list)  # SimpleRule | CompoundRule


@dataclass
class RuleSetModel(Model):
    criterion: str = "firstHit"  # first RuleSelectionMethod: firstHit | weightedSum | weightedMax
    default_score: Optional[str] = None
    default_confidence: Optional[float] = None
    rules: List[object] = field(default_factory=list)


# naive Bayes ------------------------------------------------------------------


@dataclass
class BayesInput:
    field: str
    pair_counts: Dict[str, Dict[str, float]] = field(default_factory=dict)   # value -> {target: count}
    gaussian: Dict[str, Tuple[float, float]] = field(default_factory=dict)   # target -> (mean, variance)


@dataclass
class NaiveBayesModel(Model):
    threshold: float = 0.0
    inputs: List[BayesInput] = field(default_factory=list)
    output_field: Optional[str] = None
    target_counts: Dict[str, float] = field(default_factory=dict)  # BayesOutput, document order


# k-nearest neighbours ---------------------------------------------------------


@dataclass
class KNNInput:
    field: str
    weight: float = 1.0
    compare_function: Optional[str] = None


@dataclass
class NearestNeighborModel(Model):
    k: int = 1
    continuous_method: str = "average"
    categorical_method: str = "majorityVote"
    threshold: float = 0.001
    measure_kind: str = "distance"
    metric: str = "euclidean"
    minkowski_p: float = 2.0
    compare_function: str = "absDiff"
    inputs: List[KNNInput] = field(default_factory=list)
    instance_fields: Dict[str, str] = field(default_factory=dict)  # field -> InlineTable column
    rows: List[Dict[str, str]] = field(default_factory=list)       # InlineTable rows


# association rules ---------------------------------------------------------------


@dataclass
class AssociationRule:
    antecedent: str  # itemset id
    consequent: str  # itemset id
    support: float
    confidence: float
    lift: Optional[float] = None
    leverage: Optional[float] = None
    affinity: Optional[float] = None
    rule_id: Optional[str] = None


@dataclass
class AssociationModel(Model):
    """``AssociationModel`` (`functionName="associationRules"`): items, itemsets and rules. It has
    no target field, so the reference's target extraction yields ``EmptyScore`` for every record;
    the rules are exposed through ``ruleValue`` output fields."""

    items: Dict[str, str] = field(default_factory=dict)          # item id -> value
    itemsets: Dict[str, List[str]] = field(default_factory=dict)  # itemset id -> item ids
    rules: List[AssociationRule] = field(default_factory=list)
    number_of_transactions: int = 0
    minimum_support: float = 0.0
    minimum_confidence: float = 0.0
