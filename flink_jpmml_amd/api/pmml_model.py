"""``PmmlModel``: the model handle user UDFs receive (`S/api/PmmlModel.scala:43-176`).

Per-record API (reference parity)::

    prediction = model.predict(DenseVector(1, 1, 1, 1), replace_nan=None)   # Prediction(Score(3.0))

runs ``validate → prepare → evaluate → extract`` under a Try and never raises for a bad record
(`S/api/PmmlModel.scala:109-119`). On a model bound to a device (the operators bind every model
to the rank's GPU; ``ScoringConfig.device="auto"`` is the default) a conforming vector is scored
as a 1-row batch by the device plan; unbound models, and vectors that fail validation, run the
host float64 pipeline — the semantic reference (its tree walks in C++: ``models/native_tree.py``).

Batch API (the MI355X path)::

    scores, valid = model.predict_batch(X, device="cuda")     # X: [rows, active fields]

prepares and scores a whole micro-batch with the HIP kernels; ``valid[i] == False`` is exactly
the case where ``predict`` would return ``EmptyScore``.
"""

from __future__ import annotations

import logging
import math
from typing import Any, Dict, List, Optional, Sequence

import numpy as np

from ..domain.prediction import Prediction, Score, EmptyScore
from .converter import PmmlInput, vector_conversion
from .evaluator import EMPTY_EVALUATOR, Evaluator
from .exceptions import InputValidationException, JPMMLExtractionException
from .pipeline import FieldValue, Pipeline
from .reader import ModelReader
from .batch import PredictionBatch, RecordBatch, as_record_batch
from .vectors import Vector, as_vector, pack_vectors_masked

logger = logging.getLogger(__name__)


class PmmlModel(Pipeline):
    def __init__(self, evaluator: Evaluator):
        self.evaluator = evaluator
        self._scorer = None

    # ------------------------------------------------------------------ factories
    @staticmethod
    def from_reader(reader: ModelReader) -> "PmmlModel":
        """Read + parse + build the evaluator (`S/api/PmmlModel.scala:53-58`). Errors propagate;
        operators wrap them into :class:`ModelLoadingException`."""
        from ..runtime.compiled import CompiledPmml

        text = reader.build_distributed_path()
        return PmmlModel(Evaluator.apply(CompiledPmml.from_string(text, source=reader.source_path)))

    @staticmethod
    def from_path(path: str) -> "PmmlModel":
        return PmmlModel.from_reader(ModelReader(path))

    @staticmethod
    def from_string(text: str) -> "PmmlModel":
        from ..runtime.compiled import CompiledPmml

        return PmmlModel(Evaluator.apply(CompiledPmml.from_string(text)))

    @staticmethod
    def empty() -> "PmmlModel":
        return PmmlModel(EMPTY_EVALUATOR)

    fromReader = from_reader  # noqa: N815

    # ------------------------------------------------------------------ properties
    @property
    def compiled(self):
        return self.evaluator.model

    @property
    def model_name(self) -> Optional[str]:
        return self.evaluator.model.model_name

    modelName = model_name  # noqa: N815

    @property
    def active_fields(self) -> List[str]:
        return list(self.evaluator.model.active_fields)

    @property
    def is_empty(self) -> bool:
        return self.evaluator is EMPTY_EVALUATOR

    # ------------------------------------------------------------------ device binding
    def bind(self, device: Any = None, config: Any = None, pipeline: Any = None, plan: Any = None) -> "PmmlModel":
        """Attach the scorer that record batches go through: the HIP plan on ``device`` (shared
        ``pipeline`` of streams + input ring), or the host oracle. Operators call this once per
        subtask and model; :func:`flink_jpmml_amd.runtime.engine.make_scorer` applies the
        config's fallback policy."""
        if not self.is_empty:
            from ..runtime.engine import make_scorer

            self._scorer = make_scorer(self.evaluator.model, device, config, pipeline, plan)
        return self

    @property
    def scorer(self):
        if self._scorer is None and not self.is_empty:
            self.bind(None)
        return self._scorer

    @property
    def on_device(self) -> bool:
        return self._scorer is not None and getattr(self._scorer, "kind", "") == "device"

    # ------------------------------------------------------------------ per-record pipeline
    def predict(self, input_vector: Any, replace_nan: Optional[float] = None):
        """Score one vector → :class:`Prediction` (the reference's contract), or a whole
        :class:`RecordBatch` / ``[rows, fields]`` matrix → :class:`PredictionBatch` (asynchronous
        on the device; row ``i`` equals ``predict(batch.vector(i))``)."""
        batch = as_record_batch(input_vector)
        if batch is not None:
            return self.predict_records(batch, replace_nan)
        if self.on_device:
            pred = self._predict_one_device(input_vector, replace_nan)
            if pred is not None:
                return pred
        elif self._host_row_path():
            pred = self._predict_one_host(input_vector, replace_nan)
            if pred is not None:
                return pred

        def run() -> float:
            validated = self.validate_input(input_vector)
            prepared = self.prepare_input(validated, replace_nan)
            result = self.evaluate_input(prepared)
            return self.extract_target(result)

        return Prediction.extract_prediction(run)

    def _predict_one_device(self, input_vector: Any, replace_nan: Optional[float]) -> Optional[Prediction]:
        """The reference's per-record call (`S/package.scala:76-82,111-114`) on the bound device
        plan: the vector is a 1-row batch through the same kernels as a columnar batch (whose row
        ``i`` equals ``predict(batch.vector(i))``). Returns None — the caller then runs the host
        pipeline, which produces the reference's exception / EmptyScore handling — for anything
        that is not a conforming numeric vector."""
        try:
            vec = as_vector(input_vector)
        except Exception:  # noqa: BLE001 - the host path reports the validation failure
            return None
        width = len(self.evaluator.model.active_fields)
        if not isinstance(vec, Vector) or vec.size != width or not self._numeric_inputs():
            return None
        X, absent, ok = pack_vectors_masked([vec], width)
        if ok is not None and not ok[0]:
            return None
        row = X[0]
        if absent is not None and absent.any():  # sparse-absent entries: replace_nan, else missing
            row = np.where(absent[0], np.nan if replace_nan is None else replace_nan, row)
        score_row = getattr(self._scorer, "score_row", None)
        if score_row is not None:
            s, v = score_row(row)
        else:
            pb = self._scorer.submit_batch(RecordBatch(row[None, :]), None)
            s, v = float(pb.scores[0]), bool(pb.valid[0])
        return Prediction(Score(s)) if v else Prediction(EmptyScore)

    _HOOKS = ("validate_input", "prepare_input", "evaluate_input", "extract_target")

    def _numeric_inputs(self) -> bool:
        """Every active field takes a number: a vector entry for a string-typed field is a
        preparation failure per record (JPMML refuses it), while a batch would read it as a
        vocabulary code -- such models keep the per-record pipeline."""
        ok = self.__dict__.get("_numeric_ok")
        if ok is None:
            compiled = self.evaluator.model
            ok = not any(compiled.schema.is_string(n) for n in compiled.active_fields)
            self._numeric_ok = ok
        return ok

    def _host_row_path(self) -> bool:
        """The 1-row batch oracle may stand in for the per-record pipeline on the host: the model
        has an evaluator and no subclass replaced a pipeline stage (a replaced stage must run)."""
        if self.is_empty or not self._numeric_inputs():
            return False
        cls = type(self)
        ok = cls.__dict__.get("_host_row_ok")
        if ok is None:
            ok = all(getattr(cls, h) is getattr(PmmlModel, h) for h in self._HOOKS)
            setattr(cls, "_host_row_ok", ok)
        return ok

    def _predict_one_host(self, input_vector: Any, replace_nan: Optional[float]) -> Optional[Prediction]:
        """A conforming numeric vector as a 1-row batch through the float64 oracle's vectorised
        preparation and native tree walk -- the same function of the record as the per-record
        pipeline (a batch row ``i`` equals ``predict(batch.vector(i))``), about twice as fast per
        call. None (the caller runs the pipeline, which reports the reference's exceptions /
        EmptyScore) for anything else."""
        try:
            vec = as_vector(input_vector)
        except Exception:  # noqa: BLE001 - the pipeline reports the validation failure
            return None
        compiled = self.evaluator.model
        width = len(compiled.active_fields)
        if not isinstance(vec, Vector) or vec.size != width:
            return None
        X, absent, ok = pack_vectors_masked([vec], width)
        if ok is not None and not ok[0]:
            return None
        try:
            s, v = compiled.score_matrix_oracle(X, replace_nan=replace_nan, absent=absent)
        except Exception:  # noqa: BLE001 - let the pipeline produce the per-record outcome
            return None
        return Prediction(Score(float(s[0]))) if bool(v[0]) else Prediction(EmptyScore)

    def validate_input(self, v: Any) -> PmmlInput:
        """Size check against the active fields, then vector → map (`S/api/PmmlModel.scala:127-134`)."""
        model = self.evaluator.model
        vec: Vector = as_vector(v)
        size = len(model.active_fields)
        if vec.size != size:
            raise InputValidationException(f"input vector {vec!r} size {vec.size} is not conform to model size {size}")
        return vector_conversion(vec, self.evaluator)

    def prepare_input(self, input_map: PmmlInput, replace_nan: Optional[float] = None) -> Dict[str, FieldValue]:
        """Per-field preparation (`S/api/PmmlModel.scala:143-152`): absent values take
        ``replace_nan`` (if given) else PMML missing-value handling."""
        compiled = self.evaluator.model
        schema = compiled.schema
        out: Dict[str, FieldValue] = {}
        for name in compiled.active_fields:
            raw = input_map.get(name)
            if raw is None and replace_nan is not None:
                raw = replace_nan
            try:
                enc = schema.prepare_value(name, raw, compiled.mining_fields.get(name))
                df = schema.data_fields.get(name)
                fv = FieldValue(schema.decode(name, enc), enc, df.data_type if df else None, df.optype if df else None)
                outcome: Any = fv
            except Exception as e:  # noqa: BLE001 - any failure becomes InputPreparationException
                outcome = e
            k, fv = self.prepare_and_emit(outcome, name)
            out[k] = fv
        return out

    def evaluate_input(self, prepared: Dict[str, FieldValue]) -> Dict[str, Any]:
        """Evaluate one prepared record; returns ``{target fields..., output fields...}`` decoded."""
        compiled = self.evaluator.model
        row = np.array([[prepared[name].encoded if name in prepared else math.nan
                         for name in compiled.active_fields]], dtype=np.float64)
        res, outs = compiled.evaluate_prepared(row)
        result: Dict[str, Any] = {}
        labels = res.label_strings()
        for tf in compiled.target_fields:
            if not res.valid[0]:
                result[tf] = None
            elif res.kind == "regression":
                result[tf] = float(res.value[0])
            else:
                result[tf] = labels[0]
        for k, v in outs.items():
            result[k] = compiled.schema.decode(k, float(v[0]))
        return result

    def extract_target(self, evaluation_result: Dict[str, Any]) -> float:
        """First named target → double, else :class:`JPMMLExtractionException`
        (`S/api/PmmlModel.scala:167-174`)."""
        targets = self.extract_target_fields(evaluation_result)
        if targets:
            v = self.extract_target_value(targets[0][1])
            if v is not None:
                return v
        raise JPMMLExtractionException("Target value is null.")

    def outputs_of(self, evaluation_result: Dict[str, Any]) -> Dict[str, Any]:
        return dict(self.extract_output_fields(evaluation_result))

    def predict_with_outputs(self, input_vector: Any, replace_nan: Optional[float] = None) -> Prediction:
        """Like :meth:`predict` but also returns the PMML ``<Output>`` fields in
        ``Prediction.outputs`` (the reference extracts and drops them)."""
        try:
            validated = self.validate_input(input_vector)
            prepared = self.prepare_input(validated, replace_nan)
            result = self.evaluate_input(prepared)
        except Exception as e:  # noqa: BLE001
            return Prediction.on_failed_prediction(e)
        outputs = self.outputs_of(result)
        try:
            target = self.extract_target(result)
        except Exception as e:  # noqa: BLE001 - no / null target: EmptyScore, outputs still reported
            empty = Prediction.on_failed_prediction(e)
            return Prediction(empty.value, outputs)  # (e.g. AssociationModel: rules, no target field)
        return Prediction(Score(target), outputs)

    # Scala-style aliases
    validateInput = validate_input  # noqa: N815
    prepareInput = prepare_input  # noqa: N815
    evaluateInput = evaluate_input  # noqa: N815
    extractTarget = extract_target  # noqa: N815

    # ------------------------------------------------------------------ batch API
    def predict_records(self, batch: RecordBatch, replace_nan: Optional[float] = None,
                        keep_device: bool = False) -> PredictionBatch:
        """Columnar ``predict``: validation (row width), preparation, evaluation and extraction for
        a whole batch on the bound scorer. Never raises for bad records: rows the per-record path
        would score as ``EmptyScore`` are invalid in the result."""
        n = len(batch)
        if self.is_empty:  # EmptyEvaluatorException for every record -> EmptyScore
            return PredictionBatch.empty(n)
        width = len(self.evaluator.model.active_fields)
        if batch.n_features != width:  # InputValidationException for every record
            logger.warning("Error while validate input: batch width %d is not conform to model size %d",
                           batch.n_features, width)
            return PredictionBatch.empty(n)
        return self.scorer.submit_batch(batch, replace_nan, keep_device=keep_device)

    def predict_batch(self, X: Any, replace_nan: Optional[float] = None, device: Any = None, **opts):
        """Score a ``[rows, active_fields]`` matrix (numpy or torch; NaN = missing) or a sequence
        of vectors. Returns ``(scores, valid)``; numpy on host, torch tensors on device."""
        compiled = self.evaluator.model
        if isinstance(X, (list, tuple)) and X and isinstance(as_vector(X[0]), Vector) and not np.isscalar(X[0]):
            return self.predict_vectors(X, replace_nan, device, **opts)
        return compiled.score_matrix(X, replace_nan=replace_nan, device=device, **opts)

    def predict_vectors(self, vectors: Sequence[Any], replace_nan: Optional[float] = None, device: Any = None,
                        **opts) -> List[Prediction]:
        """Batch version of :meth:`predict` over vector objects → list of :class:`Prediction`."""
        compiled = self.evaluator.model
        width = len(compiled.active_fields)
        X, absent, ok_size = pack_vectors_masked(vectors, width)
        # replace_nan fills only the entries sparse vectors do not store (per-record parity)
        scores, valid = compiled.score_matrix(X, replace_nan=replace_nan, device=device, absent=absent, **opts)
        if not isinstance(scores, np.ndarray):
            scores = scores.detach().cpu().numpy()
            valid = valid.detach().cpu().numpy()
        valid = np.asarray(valid, dtype=bool) if ok_size is None else np.asarray(valid, dtype=bool) & ok_size
        return [Prediction(Score(float(s))) if v else Prediction(EmptyScore) for s, v in zip(scores, valid)]

    def __repr__(self) -> str:
        return f"PmmlModel({self.evaluator!r})"
