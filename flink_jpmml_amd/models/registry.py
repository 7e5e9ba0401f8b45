"""Model-element → evaluator registry (the analogue of JPMML's ``ModelEvaluatorFactory``,
`S/api/PmmlModel.scala:45`)."""

from __future__ import annotations

from typing import Callable, Dict

from ..api.exceptions import UnsupportedFeatureException
from ..pmml import ir
from ..pmml.fields import FieldSchema
from .base import ModelEvaluator


def _registry() -> Dict[type, Callable[..., ModelEvaluator]]:
    from .association import AssociationEvaluator
    from .clustering import ClusteringEvaluator
    from .knn import NearestNeighborEvaluator
    from .mining import MiningEvaluator
    from .naive_bayes import NaiveBayesEvaluator
    from .neural import NeuralEvaluator
    from .regression import GeneralRegressionEvaluator, RegressionEvaluator
    from .svm import SvmEvaluator
    from .scorecard import make_ruleset_evaluator, make_scorecard_evaluator
    from .tree import TreeEvaluator

    return {
        ir.ClusteringModel: ClusteringEvaluator,
        ir.TreeModel: TreeEvaluator,
        ir.MiningModel: MiningEvaluator,
        ir.RegressionModel: RegressionEvaluator,
        ir.GeneralRegressionModel: GeneralRegressionEvaluator,
        ir.NeuralNetwork: NeuralEvaluator,
        ir.SupportVectorMachineModel: SvmEvaluator,
        ir.Scorecard: make_scorecard_evaluator,
        ir.RuleSetModel: make_ruleset_evaluator,
        ir.NaiveBayesModel: NaiveBayesEvaluator,
        ir.NearestNeighborModel: NearestNeighborEvaluator,
        ir.AssociationModel: AssociationEvaluator,
    }


_REG: Dict[type, Callable[..., ModelEvaluator]] = {}


def make_evaluator(model: ir.Model, schema: FieldSchema) -> ModelEvaluator:
    global _REG
    if not _REG:
        _REG = _registry()
    cls = _REG.get(type(model))
    if cls is None:
        raise UnsupportedFeatureException(f"no evaluator for {type(model).__name__}")
    return cls(model, schema)
