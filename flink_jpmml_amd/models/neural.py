"""NeuralNetwork (multi-layer perceptron) — oracle and dense-layer lowering.

``NeuralInputs`` derive each input (usually ``NormContinuous``/``NormDiscrete``); every
``NeuralLayer`` computes ``z = W·a + bias`` then an activation (``logistic``, ``tanh``,
``identity``, ``rectifier``, ``exponential``, ``reciprocal``, ``square``, ``Gauss``, ``sine``,
``cosine``, ``Elliott``, ``arctan``, ``threshold``, ``radialBasis``) and an optional layer
normalisation (``softmax``/``simplemax``). ``NeuralOutputs`` map neurons back to the target:
``NormContinuous`` (inverse) / ``FieldRef`` for regression, ``NormDiscrete`` for class
probabilities.

:meth:`NeuralEvaluator.dense_layers` lowers a strictly layered network into ``[(W, b, act,
norm)]`` — the operand list of the fused bf16 MFMA MLP kernel.
"""

from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import numpy as np

from ..api.exceptions import UnsupportedFeatureException
from ..pmml import ir
from ..pmml.fields import NAN, Columns, FieldSchema, denorm_continuous, eval_expression
from .base import ModelEvaluator, ModelResult

ACTIVATIONS = ("threshold", "logistic", "tanh", "identity", "exponential", "reciprocal", "square", "Gauss",
               "sine", "cosine", "Elliott", "arctan", "rectifier")


def activate(name: str, z: np.ndarray, threshold: float = 0.0) -> np.ndarray:
    with np.errstate(over="ignore", divide="ignore", invalid="ignore"):
        if name == "logistic":
            return 1.0 / (1.0 + np.exp(-z))
        if name == "tanh":
            return np.tanh(z)
        if name == "identity":
            return z
        if name == "rectifier":
            return np.maximum(z, 0.0)
        if name == "exponential":
            return np.exp(z)
        if name == "reciprocal":
            return 1.0 / z
        if name == "square":
            return z * z
        if name == "Gauss":
            return np.exp(-z * z)
        if name == "sine":
            return np.sin(z)
        if name == "cosine":
            return np.cos(z)
        if name == "Elliott":
            return z / (1.0 + np.abs(z))
        if name == "arctan":
            return 2.0 * np.arctan(z) / np.pi
        if name == "threshold":
            return (z > threshold).astype(np.float64)
    raise UnsupportedFeatureException(f"activationFunction {name!r}")


def normalize_layer(name: Optional[str], A: np.ndarray) -> np.ndarray:
    if name in (None, "none"):
        return A
    if name == "softmax":
        Z = A - A.max(axis=1, keepdims=True)
        E = np.exp(Z)
        return E / E.sum(axis=1, keepdims=True)
    if name == "simplemax":
        return A / A.sum(axis=1, keepdims=True)
    raise UnsupportedFeatureException(f"layer normalizationMethod {name!r}")


class NeuralEvaluator(ModelEvaluator):
    def __init__(self, model: ir.NeuralNetwork, schema: FieldSchema):
        super().__init__(model, schema)
        self.nn = model
        for inp in model.inputs:
            schema.types.setdefault(inp.derived.name or f"__in_{inp.id}", "double")
        if self.kind == "classification":
            cats: List[str] = []
            for o in model.outputs:
                ex = o.derived.expression
                if isinstance(ex, ir.NormDiscrete) and ex.value not in cats:
                    cats.append(ex.value)
            decl = self.classification_categories()
            self.categories = [c for c in decl if c in cats] + [c for c in cats if c not in decl]
        else:
            self.categories = None

    # ------------------------------------------------------------------ structure
    def _layer_params(self, layer: ir.NeuralLayer) -> Tuple[str, float, Optional[str]]:
        act = layer.activation or self.nn.activation
        thr = layer.threshold if layer.threshold is not None else self.nn.threshold
        norm = layer.normalization or self.nn.normalization
        return act, thr, norm

    def dense_layers(self) -> List[Tuple[np.ndarray, np.ndarray, str, float, Optional[str]]]:
        """Lower to ``[(W[in, out], b[out], activation, threshold, normalization)]``; raises
        :class:`UnsupportedFeatureException` when connections skip layers."""
        prev_ids = [inp.id for inp in self.nn.inputs]
        out = []
        for layer in self.nn.layers:
            act, thr, norm = self._layer_params(layer)
            if act == "radialBasis":
                raise UnsupportedFeatureException("radialBasis layers are not lowered to dense GEMMs")
            idx = {nid: i for i, nid in enumerate(prev_ids)}
            W = np.zeros((len(prev_ids), len(layer.neurons)))
            b = np.zeros(len(layer.neurons))
            for j, neu in enumerate(layer.neurons):
                b[j] = neu.bias
                for src, w in neu.connections:
                    if src not in idx:
                        raise UnsupportedFeatureException("connection skips a layer")
                    W[idx[src], j] += w
            out.append((W, b, act, thr, norm))
            prev_ids = [n.id for n in layer.neurons]
        return out

    def input_columns(self, cols: Columns) -> np.ndarray:
        mats = []
        for inp in self.nn.inputs:
            mats.append(eval_expression(inp.derived.expression, cols))
        return np.stack(mats, axis=1)

    # ------------------------------------------------------------------ oracle
    def _native_layers(self) -> List[Optional[Tuple[np.ndarray, np.ndarray, np.ndarray]]]:
        """Per layer ``(order, W, b)`` for the native ``seq_affine`` when every neuron reads the
        previous layer's neurons (or the inputs) in one shared connection order, else None."""
        cached = getattr(self, "_native", None)
        if cached is not None:
            return cached
        from ..native import fastpath

        fp = fastpath()
        out: List[Optional[Tuple[np.ndarray, np.ndarray, np.ndarray]]] = []
        prev_ids = [inp.id for inp in self.nn.inputs]
        for layer in self.nn.layers:
            act, _, _ = self._layer_params(layer)
            idx = {nid: i for i, nid in enumerate(prev_ids)}
            entry = None
            if fp is not None and hasattr(fp, "seq_affine") and act != "radialBasis" and layer.neurons:
                srcs = [s for s, _ in layer.neurons[0].connections]
                if all(src in idx for src in srcs) and all(
                        len(neu.connections) == len(srcs) and all(c[0] == s for c, s in zip(neu.connections, srcs))
                        for neu in layer.neurons):
                    W = np.array([[w for _, w in neu.connections] for neu in layer.neurons],
                                 dtype=np.float64).T.copy() if srcs else np.zeros((0, len(layer.neurons)))
                    entry = (np.array([idx[s] for s in srcs], dtype=np.int32), np.ascontiguousarray(W),
                             np.array([neu.bias for neu in layer.neurons], dtype=np.float64))
            out.append(entry)
            prev_ids = [n.id for n in layer.neurons]
        self._native = out
        return out

    def forward(self, A0: np.ndarray) -> Dict[str, np.ndarray]:
        vals: Dict[str, np.ndarray] = {inp.id: A0[:, i] for i, inp in enumerate(self.nn.inputs)}
        n = A0.shape[0]
        native = self._native_layers()
        prev = [inp.id for inp in self.nn.inputs]
        for li, layer in enumerate(self.nn.layers):
            act, thr, norm = self._layer_params(layer)
            if native[li] is not None and n:
                from ..native import fastpath

                order, W, b = native[li]
                Ap = np.ascontiguousarray(np.stack([vals[i] for i in prev], axis=1), dtype=np.float64)
                Z = np.empty((n, len(layer.neurons)))
                fastpath().seq_affine(Ap, Ap.shape[1], order, W, b, Z)
                A = activate(act, Z, thr)
                A = normalize_layer(norm, A)
                for j, neu in enumerate(layer.neurons):
                    vals[neu.id] = A[:, j]
                prev = [neu.id for neu in layer.neurons]
                continue
            prev = [neu.id for neu in layer.neurons]
            Z = np.zeros((n, len(layer.neurons)))
            for j, neu in enumerate(layer.neurons):
                if act == "radialBasis":
                    width = neu.width if neu.width is not None else (layer.width or self.nn.width)
                    alt = neu.altitude if neu.altitude is not None else (layer.altitude or self.nn.altitude)
                    s = np.zeros(n)
                    for src, w in neu.connections:
                        s += (vals[src] - w) ** 2
                    s = s / (2.0 * width * width)
                    fan_in = len(neu.connections)
                    Z[:, j] = np.exp(fan_in * np.log(alt) - s)
                else:
                    z = np.full(n, neu.bias)
                    for src, w in neu.connections:
                        z = z + w * vals[src]
                    Z[:, j] = z
            A = Z if act == "radialBasis" else activate(act, Z, thr)
            A = normalize_layer(norm, A)
            for j, neu in enumerate(layer.neurons):
                vals[neu.id] = A[:, j]
        return vals

    def _evaluate(self, cols: Columns) -> ModelResult:
        A0 = self.input_columns(cols)
        miss = np.any(np.isnan(A0), axis=1)
        vals = self.forward(np.nan_to_num(A0))
        return self.finish(vals, ~miss)

    def output_neurons(self) -> List[str]:
        return [o.neuron for o in self.nn.outputs]

    def finish(self, vals: Dict[str, np.ndarray], valid: np.ndarray) -> ModelResult:
        n = valid.shape[0]
        if self.kind == "classification":
            P = np.zeros((n, len(self.categories)))
            for o in self.nn.outputs:
                ex = o.derived.expression
                if isinstance(ex, ir.NormDiscrete):
                    P[:, self.categories.index(ex.value)] = vals[o.neuron]
            lab = np.argmax(P, axis=1).astype(np.float64)
            return ModelResult("classification", np.where(valid, lab, NAN), valid.copy(), categories=self.categories,
                               probs=np.where(valid[:, None], P, NAN))
        o = self.nn.outputs[0]
        y = vals[o.neuron]
        ex = o.derived.expression
        if isinstance(ex, ir.NormContinuous):
            y = denorm_continuous(ex, y)
        elif not isinstance(ex, ir.FieldRef):
            raise UnsupportedFeatureException("regression NeuralOutput must be NormContinuous or FieldRef")
        ok = valid & np.isfinite(y)
        return ModelResult("regression", np.where(ok, y, NAN), ok)
