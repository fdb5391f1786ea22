"""RPC semantics of PredictionService + ModelService over raw request bytes.

Each handler takes the serialized request and returns the serialized
response, raising :class:`~.errors.ServingError` for non-OK statuses, so any
transport (grpcio adapter, the native HTTP/2 front end, REST) can sit on top.
Behaviour follows the contract derived in SURVEY.md §2.3 from the reference
client call sites:

* Predict (``src/lib.rs:213-267``): version unset -> latest; empty
  signature_name -> ``serving_default``; inputs are signature *aliases*;
  empty output_filter -> all outputs; the effective model_spec is echoed.
  Hot path decode/encode is the native codec (zero-copy float_val views).
* GetModelMetadata (``src/lib.rs:300-312``): only ``signature_def`` is
  supported; value is ``Any(SignatureDefMap)``.
* Classify / Regress / MultiInference: tf.Example inputs (``input.proto``),
  which the reference only half-implements (``src/lib.rs:195`` panics).
* GetModelStatus / HandleReloadConfigRequest (``src/lib.rs:287-334``).
"""
from __future__ import annotations

import logging
import time
from typing import Dict, List, Optional, Sequence

import numpy as np

from .. import native
from ..schema import Any, serving, tf
from ..utils import tensors as T
from ..utils import roctx
from . import errors as E
from .manager import ModelManager
from .servable import CLASSIFY_METHOD, PREDICT_METHOD, REGRESS_METHOD

log = logging.getLogger("tfserve.core")

METHOD_PREFIX_P = "/tensorflow.serving.PredictionService/"
METHOD_PREFIX_M = "/tensorflow.serving.ModelService/"


def _spec_from_msg(ms):
    version = ms.version.value if ms.HasField("version") else None
    label = ms.version_label if ms.WhichOneof("version_choice") == "version_label" else None
    return ms.name, version, label, ms.signature_name


def _fill_spec(dst, name: str, version: int, sig: Optional[str]):
    dst.name = name
    dst.version.value = version
    if sig is not None:
        dst.signature_name = sig


class ServingCore:
    def __init__(self, manager: ModelManager, batcher=None, request_logger=None, metrics=None):
        self.manager = manager
        self.batcher = batcher
        self.request_logger = request_logger
        self.metrics = metrics
        self.replicas = None          # parallel.replicas.ReplicaControl when serving N GPU replicas
        self.tracer = None            # utils.tracing.Tracer (--trace_dir)
        self.health = None            # server.health.HealthMonitor (device-failure detection)
        self.handlers = {
            METHOD_PREFIX_P + "Predict": self.predict,
            METHOD_PREFIX_P + "Classify": self.classify,
            METHOD_PREFIX_P + "Regress": self.regress,
            METHOD_PREFIX_P + "MultiInference": self.multi_inference,
            METHOD_PREFIX_P + "GetModelMetadata": self.get_model_metadata,
            METHOD_PREFIX_M + "GetModelStatus": self.get_model_status,
            METHOD_PREFIX_M + "HandleReloadConfigRequest": self.handle_reload_config,
        }

    def handle(self, method: str, request: bytes) -> bytes:
        fn = self.handlers.get(method)
        if fn is None:
            raise E.unimplemented(f"Method not found: {method}")
        t0 = time.perf_counter()
        code = E.OK
        try:
            with roctx.range("tfs.rpc " + method.rsplit("/", 1)[-1]):
                return fn(request)
        except E.ServingError as e:
            code = e.code
            raise
        except Exception as e:   # never leak a Python traceback over the wire
            code = E.INTERNAL
            log.exception("internal error in %s", method)
            raise E.internal(f"{type(e).__name__}: {e}") from None
        finally:
            t1 = time.perf_counter()
            if self.metrics is not None:
                self.metrics.observe_rpc(method, code, t1 - t0)
            if self.tracer is not None:
                end = time.monotonic() * 1e6
                self.tracer.rpc(method, end - (t1 - t0) * 1e6, end, code)

    # ------------------------------------------------------------------ helpers
    def _resolve(self, name, version, label):
        return self.manager.resolve(name, version, label)

    def _run(self, servable, sig_name: str, inputs: Dict, out_aliases: Sequence[str]):
        if self.health is None:
            return self._run_raw(servable, sig_name, inputs, out_aliases)
        try:
            out = self._run_raw(servable, sig_name, inputs, out_aliases)
        except BaseException as e:
            from .health import is_device_failure
            # one failed batch fails every request in it with the SAME error
            # object (server/batching.py): count the batch once, not per request
            if is_device_failure(e) and not getattr(e, "_health_counted", False):
                try:
                    e._health_counted = True
                except AttributeError:
                    pass
                self.health.record(getattr(servable, "name", "?"), getattr(servable, "version", 0), False, str(e))
            raise
        self.health.record(getattr(servable, "name", "?"), getattr(servable, "version", 0), True)
        return out

    def _run_raw(self, servable, sig_name: str, inputs: Dict, out_aliases: Sequence[str]):
        if self.batcher is not None:
            return self.batcher.run(servable, sig_name, inputs, list(out_aliases))
        fault = getattr(servable, "fault", None)
        if fault is not None:
            fault.check()
        return servable.run(sig_name, inputs, list(out_aliases))

    @staticmethod
    def _check_inputs(sig, inputs: Dict[str, np.ndarray], dtypes: Dict[str, int]):
        expected = set(sig.inputs.keys())
        got = set(inputs)
        for a in sorted(got):
            if a not in expected:
                raise E.invalid(f"input tensor alias not found in signature: {a}. "
                                f"Inputs expected to be in the set {{{','.join(sorted(expected))}}}.")
        if got != expected:
            missing = sorted(expected - got)
            raise E.invalid(f"input size does not match signature: {len(got)}!={len(expected)} "
                            f"len({{{','.join(sorted(got))}}}) != len({{{','.join(sorted(expected))}}}). "
                            f"Sent extra: {{}}. Missing but required: {{{','.join(missing)}}}.")
        for i, a in enumerate(sorted(got)):
            ti = sig.inputs[a]
            dt = dtypes.get(a)
            if dt is not None and ti.dtype and dt != ti.dtype:
                raise E.invalid(f"Expects arg[{i}] to be {_dtname(ti.dtype)} but {_dtname(dt)} is provided")
            if not ti.tensor_shape.unknown_rank and len(ti.tensor_shape.dim):
                want = [d.size for d in ti.tensor_shape.dim]
                shp = list(inputs[a].shape)
                if len(shp) != len(want) or any(w >= 0 and w != s for w, s in zip(want, shp)):
                    raise E.invalid(f"input tensor alias {a}: shape {shp} is incompatible with the "
                                    f"signature shape {want}")

    # ------------------------------------------------------------------ Predict
    def predict(self, request: bytes) -> bytes:
        try:
            spec, inputs, out_filter, dtypes = native.decode_predict_request(request)
        except (native.WireError, T.TensorError) as e:
            raise E.invalid(str(e)) from None
        if spec is None:
            raise E.invalid("Missing ModelSpec")
        name, version, label, sig = spec[0].decode(), spec[1], \
            None if spec[2] is None else spec[2].decode(), spec[3].decode()
        servable = self._resolve(name, version, label)
        try:
            sig_name, sigdef = servable.signature(sig)
            self._check_inputs(sigdef, inputs, dtypes)
            outs_avail = sigdef.outputs
            if out_filter:
                seen = set()
                for a in out_filter:
                    if a not in outs_avail:
                        raise E.invalid(f"output tensor alias not found in signature: {a} Outputs expected "
                                        f"to be in the set {{{','.join(sorted(outs_avail.keys()))}}}.")
                    if a in seen:
                        raise E.invalid(f"duplicate output tensor alias: {a}")
                    seen.add(a)
                out_aliases = list(out_filter)
            else:
                out_aliases = sorted(outs_avail.keys())
            outputs = self._run(servable, sig_name, inputs, out_aliases)
            out_dt = {a: outs_avail[a].dtype for a in out_aliases}
            for a, v in outputs.items():
                if out_dt[a] == T.DT_BFLOAT16 and v.dtype != np.uint16:
                    out_dt[a] = T.dt_of(v)
            resp = native.encode_predict_response(
                native.spec_tuple(name, servable.version, None, sig_name), outputs, out_dt)
        finally:
            servable.release()
        if self.request_logger is not None:
            self.request_logger.log("predict", name, request, resp)
        return resp

    # ------------------------------------------------------------------ tf.Example paths
    @staticmethod
    def _examples(inp) -> List[bytes]:
        kind = inp.WhichOneof("kind")
        if kind == "example_list":
            exs = list(inp.example_list.examples)
            ctx = None
        elif kind == "example_list_with_context":
            exs = list(inp.example_list_with_context.examples)
            ctx = inp.example_list_with_context.context
        else:
            raise E.invalid("Input is empty")
        if not exs:
            raise E.invalid("Input is empty")
        out = []
        for ex in exs:
            if ctx is not None:
                merged = tf.Example()
                merged.CopyFrom(ctx)
                merged.MergeFrom(ex)      # example features override context ones
                for k, f in ex.features.feature.items():
                    merged.features.feature[k].CopyFrom(f)
                out.append(merged.SerializeToString())
            else:
                out.append(ex.SerializeToString())
        return out

    def _example_run(self, servable, sig_name, sigdef, examples, out_aliases):
        if "inputs" not in sigdef.inputs or len(sigdef.inputs) != 1:
            raise E.invalid(f"Expected one input Tensor for signature {sig_name} with key 'inputs'")
        if sigdef.inputs["inputs"].dtype != T.DT_STRING:
            raise E.invalid("Classification/Regression input must be DT_STRING (serialized tf.Example)")
        arr = np.empty(len(examples), dtype=object)
        arr[:] = examples
        return servable.run(sig_name, {"inputs": arr}, out_aliases)

    @staticmethod
    def _classification_result(sig_name, sigdef, outs, n) -> "serving.ClassificationResult":
        res = serving.ClassificationResult()
        classes = outs.get("classes")
        scores = outs.get("scores")
        if classes is not None:
            classes = np.asarray(classes).reshape(n, -1) if classes.size else classes.reshape(n, 0)
        if scores is not None:
            if scores.ndim not in (1, 2) or scores.shape[0] != n:
                raise E.invalid(f"Expected Tensor shape: [{n} num_classes] but got {list(scores.shape)}")
            scores = scores.reshape(n, -1)
        if classes is not None and scores is not None and classes.shape != scores.shape:
            raise E.invalid(f"Tensors class and score should match in shape. Class shape: "
                            f"{list(classes.shape)} Score shape: {list(scores.shape)}")
        k = (classes if classes is not None else scores).shape[1]
        for i in range(n):
            c = res.classifications.add()
            for j in range(k):
                cl = c.classes.add()
                if classes is not None:
                    v = classes[i, j]
                    cl.label = v.decode() if isinstance(v, bytes) else str(v)
                if scores is not None:
                    cl.score = float(scores[i, j])
        return res

    def _classify_in(self, servable, spec_sig, inp):
        sig_name, sigdef = servable.signature(spec_sig)
        if sigdef.method_name != CLASSIFY_METHOD:
            raise E.invalid(f"Expected classification signature method_name to be {CLASSIFY_METHOD}. "
                            f"Was: {sigdef.method_name}")
        outs = [a for a in ("classes", "scores") if a in sigdef.outputs]
        if not outs:
            raise E.invalid(f"Expected classification signature outputs to contain at least one of "
                            f"classes or scores: {sig_name}")
        examples = self._examples(inp)
        res_outs = self._example_run(servable, sig_name, sigdef, examples, outs)
        return sig_name, self._classification_result(sig_name, sigdef, res_outs, len(examples))

    def _regress_in(self, servable, spec_sig, inp):
        sig_name, sigdef = servable.signature(spec_sig)
        if sigdef.method_name != REGRESS_METHOD:
            raise E.invalid(f"Expected regression signature method_name to be {REGRESS_METHOD}. "
                            f"Was: {sigdef.method_name}")
        if "outputs" not in sigdef.outputs:
            raise E.invalid(f"No regression outputs found in signature {sig_name}")
        examples = self._examples(inp)
        outs = self._example_run(servable, sig_name, sigdef, examples, ["outputs"])
        v = outs["outputs"]
        n = len(examples)
        if v.ndim == 2 and v.shape[1] == 1:
            v = v.reshape(-1)
        if v.ndim != 1 or v.shape[0] != n:
            raise E.invalid(f"Expected output Tensor shape to be either [batch_size] or [batch_size, 1] "
                            f"but got {list(outs['outputs'].shape)}")
        res = serving.RegressionResult()
        for x in v:
            res.regressions.add(value=float(x))
        return sig_name, res

    def classify(self, request: bytes) -> bytes:
        req = _parse(serving.ClassificationRequest, request)
        if not req.HasField("model_spec"):
            raise E.invalid("Missing ModelSpec")
        name, version, label, sig = _spec_from_msg(req.model_spec)
        servable = self._resolve(name, version, label)
        try:
            sig_name, res = self._classify_in(servable, sig, req.input)
            resp = serving.ClassificationResponse()
            resp.result.CopyFrom(res)
            _fill_spec(resp.model_spec, name, servable.version, sig_name)
        finally:
            servable.release()
        out = resp.SerializeToString()
        if self.request_logger is not None:
            self.request_logger.log("classify", name, request, out)
        return out

    def regress(self, request: bytes) -> bytes:
        req = _parse(serving.RegressionRequest, request)
        if not req.HasField("model_spec"):
            raise E.invalid("Missing ModelSpec")
        name, version, label, sig = _spec_from_msg(req.model_spec)
        servable = self._resolve(name, version, label)
        try:
            sig_name, res = self._regress_in(servable, sig, req.input)
            resp = serving.RegressionResponse()
            resp.result.CopyFrom(res)
            _fill_spec(resp.model_spec, name, servable.version, sig_name)
        finally:
            servable.release()
        out = resp.SerializeToString()
        if self.request_logger is not None:
            self.request_logger.log("regress", name, request, out)
        return out

    def multi_inference(self, request: bytes) -> bytes:
        req = _parse(serving.MultiInferenceRequest, request)
        if not req.tasks:
            raise E.invalid("Tasks is empty")
        names = {t.model_spec.name for t in req.tasks}
        if len(names) != 1:
            raise E.invalid("All ModelSpecs in a MultiInferenceRequest must access the same model name.")
        sigs = [t.model_spec.signature_name or "serving_default" for t in req.tasks]
        if len(set(sigs)) != len(sigs):
            raise E.invalid("Duplicate evaluation of signature: " +
                            next(s for s in sigs if sigs.count(s) > 1))
        first = req.tasks[0].model_spec
        name, version, label, _ = _spec_from_msg(first)
        servable = self._resolve(name, version, label)
        resp = serving.MultiInferenceResponse()
        try:
            for t in req.tasks:
                r = resp.results.add()
                if t.method_name == CLASSIFY_METHOD:
                    sig_name, res = self._classify_in(servable, t.model_spec.signature_name, req.input)
                    r.classification_result.CopyFrom(res)
                elif t.method_name == REGRESS_METHOD:
                    sig_name, res = self._regress_in(servable, t.model_spec.signature_name, req.input)
                    r.regression_result.CopyFrom(res)
                else:
                    raise E.unimplemented(f"Unsupported signature method_name: {t.method_name}")
                _fill_spec(r.model_spec, name, servable.version, sig_name)
        finally:
            servable.release()
        return resp.SerializeToString()

    # ------------------------------------------------------------------ metadata / status
    def get_model_metadata(self, request: bytes) -> bytes:
        req = _parse(serving.GetModelMetadataRequest, request)
        if not req.HasField("model_spec"):
            raise E.invalid("Missing ModelSpec")
        if not req.metadata_field:
            raise E.invalid("GetModelMetadataRequest must specify at least one metadata_field")
        for f in req.metadata_field:
            if f != "signature_def":
                raise E.invalid(f"Metadata field {f} is not supported")
        name, version, label, _sig = _spec_from_msg(req.model_spec)
        servable = self._resolve(name, version, label)
        try:
            sdm = serving.SignatureDefMap()
            for k, v in servable.signatures.items():
                sdm.signature_def[k].CopyFrom(v)
            resp = serving.GetModelMetadataResponse()
            _fill_spec(resp.model_spec, name, servable.version, None)
            resp.metadata["signature_def"].Pack(sdm)
        finally:
            servable.release()
        return resp.SerializeToString()

    def get_model_status(self, request: bytes) -> bytes:
        req = _parse(serving.GetModelStatusRequest, request)
        if not req.HasField("model_spec"):
            raise E.invalid("Missing ModelSpec")
        name, version, label, _ = _spec_from_msg(req.model_spec)
        if label is not None:
            cfg = self.manager.model_config(name)
            if cfg is None or label not in cfg.version_labels:
                raise E.invalid(f"Unrecognized servable version label: {label}")
            version = cfg.version_labels[label]
        resp = serving.GetModelStatusResponse()
        for vs in self.manager.status(name, version):
            m = resp.model_version_status.add(version=vs.version, state=vs.state)
            m.status.error_code = vs.error_code
            m.status.error_message = vs.error_message
        return resp.SerializeToString()

    def handle_reload_config(self, request: bytes) -> bytes:
        req = _parse(serving.ReloadConfigRequest, request)
        resp = serving.ReloadConfigResponse()
        if self.replicas is not None:
            # validate here (fail fast, nothing published), then apply on every replica
            self.manager.validate_config(req.config)
            errs = self.replicas.reload(req.config)
        else:
            errs = self.manager.apply_config(req.config, wait=True)
        if errs:
            resp.status.error_code = errs[0].code
            resp.status.error_message = "; ".join(e.message for e in errs)
        else:
            resp.status.error_code = E.OK
        return resp.SerializeToString()


def _parse(cls, data: bytes):
    try:
        return cls.FromString(data)
    except Exception as e:
        raise E.invalid(f"failed to parse {cls.DESCRIPTOR.name}: {e}") from None


def _dtname(dt: int) -> str:
    n = T.DT_NAMES.get(dt, str(dt))
    return {"DT_FLOAT": "float", "DT_DOUBLE": "double", "DT_INT32": "int32", "DT_INT64": "int64",
            "DT_STRING": "string", "DT_BOOL": "bool", "DT_UINT8": "uint8", "DT_HALF": "half",
            "DT_BFLOAT16": "bfloat16"}.get(n, n.lower())
