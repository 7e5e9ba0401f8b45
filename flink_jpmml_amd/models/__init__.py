"""PMML model families: float64 host oracle + lowering to device layouts.

| family | PMML element | oracle | device kernel |
|---|---|---|---|
| clustering | ``ClusteringModel`` | :mod:`.clustering` | ``cluster_argmin`` (HIP) |
| trees / ensembles | ``TreeModel``, ``MiningModel`` | :mod:`.tree`, :mod:`.mining` | ``tree_ensemble`` (HIP) |
| regression | ``RegressionModel``, ``GeneralRegressionModel`` | :mod:`.regression` | ``linear_link`` (HIP) |
| neural network | ``NeuralNetwork`` | :mod:`.neural` | ``mlp_bf16`` (HIP, MFMA) |
| SVM | ``SupportVectorMachineModel`` | :mod:`.svm` | ``svm_kernel`` (HIP) |
"""

from .base import ModelEvaluator, ModelResult, result_scores
from .registry import make_evaluator

__all__ = ["ModelEvaluator", "ModelResult", "make_evaluator", "result_scores"]
