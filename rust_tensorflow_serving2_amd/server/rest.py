"""TF-Serving-compatible REST API (the container's port 8501, which the
reference maps to host 9001 in ``serving/rundocker.sh:15`` but never calls).

Routes (JSON in/out, same shapes as TensorFlow Serving's REST API):

* ``GET  /v1/models/<name>[/versions/<v>|/labels/<l>]``          -> model status
* ``GET  /v1/models/<name>[/versions/<v>|/labels/<l>]/metadata`` -> signature_def map
* ``POST /v1/models/<name>[...]:predict``   row (``instances``) or columnar (``inputs``) format
* ``POST /v1/models/<name>[...]:classify`` / ``:regress``  (``examples`` + optional ``context``)
* ``GET  /monitoring/prometheus/metrics``   Prometheus text (utils/metrics.py)

Every route is translated into the same serialized gRPC request and handed to
:class:`~.core.ServingCore`, so REST and gRPC share one implementation of the
RPC semantics.  Binary strings use ``{"b64": "..."}``.  The listening socket is
bound with ``SO_REUSEPORT`` so every GPU replica can share the port.
"""
from __future__ import annotations

import base64
import json
import logging
import re
import socket
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Dict, Optional, Tuple

import numpy as np

from .. import native
from ..schema import serving, tf
from ..utils import tensors as T
from . import errors as E

log = logging.getLogger("tfserve.rest")

_ROUTE = re.compile(r"^/v1/models/(?P<name>[^/:]+)"
                    r"(?:/versions/(?P<version>-?\d+)|/labels/(?P<label>[^/:]+))?"
                    r"(?P<rest>/metadata|:predict|:classify|:regress)?/?$")

HTTP_STATUS = {E.OK: 200, E.CANCELLED: 499, E.UNKNOWN: 500, E.INVALID_ARGUMENT: 400,
               E.DEADLINE_EXCEEDED: 504, E.NOT_FOUND: 404, E.ALREADY_EXISTS: 409,
               E.PERMISSION_DENIED: 403, E.RESOURCE_EXHAUSTED: 429, E.FAILED_PRECONDITION: 400,
               E.ABORTED: 409, E.OUT_OF_RANGE: 400, E.UNIMPLEMENTED: 501, E.INTERNAL: 500,
               E.UNAVAILABLE: 503, E.DATA_LOSS: 500, E.UNAUTHENTICATED: 401}

STATE_NAMES = {0: "UNKNOWN", 10: "START", 20: "LOADING", 30: "AVAILABLE", 40: "UNLOADING", 50: "END"}


# ---------------------------------------------------------------- JSON <-> tensors
def _decode_value(v):
    if isinstance(v, dict):
        if set(v) == {"b64"}:
            return base64.b64decode(v["b64"])
        raise E.invalid("JSON object where a tensor value was expected (only {\"b64\": ...} is allowed)")
    if isinstance(v, list):
        return [_decode_value(x) for x in v]
    return v


def json_to_array(value, dtype: int) -> np.ndarray:
    v = _decode_value(value)
    if dtype == T.DT_STRING:
        arr = np.array(v, dtype=object)
        flat = arr.reshape(-1)
        for i, x in enumerate(flat):
            flat[i] = x if isinstance(x, bytes) else str(x).encode()
        return arr
    npdt = T.np_dtype(dtype) if dtype else None
    try:
        arr = np.array(v, dtype=npdt)
    except (ValueError, TypeError) as e:
        raise E.invalid(f"Failed to process element: {e}") from None
    if arr.dtype == object:
        raise E.invalid("JSON value is a ragged list (all elements of a tensor must have the same shape)")
    return arr


def array_to_json(a: np.ndarray):
    if a.dtype == object:
        def enc(x):
            if isinstance(x, bytes):
                try:
                    return x.decode("utf-8")
                except UnicodeDecodeError:
                    return {"b64": base64.b64encode(x).decode()}
            return x
        return np.vectorize(enc, otypes=[object])(a).tolist() if a.size else a.tolist()
    return a.tolist()


def feature_from_json(v) -> "tf.Feature":
    f = tf.Feature()
    vals = v if isinstance(v, list) else [v]
    vals = [_decode_value(x) for x in vals]
    if not vals:
        f.float_list.SetInParent()
    elif all(isinstance(x, bytes) for x in vals) or all(isinstance(x, str) for x in vals):
        f.bytes_list.value.extend(x if isinstance(x, bytes) else x.encode() for x in vals)
    elif all(isinstance(x, int) and not isinstance(x, bool) for x in vals):
        f.int64_list.value.extend(vals)
    elif all(isinstance(x, (int, float)) for x in vals):
        f.float_list.value.extend(float(x) for x in vals)
    else:
        raise E.invalid(f"unsupported feature value {v!r}")
    return f


def example_from_json(obj: dict) -> "tf.Example":
    if not isinstance(obj, dict):
        raise E.invalid("each example must be a JSON object of feature name -> value(s)")
    ex = tf.Example()
    for k, v in obj.items():
        ex.features.feature[k].CopyFrom(feature_from_json(v))
    return ex


# ---------------------------------------------------------------- request translation
class RestHandler:
    """Transport-independent REST semantics (unit-testable without sockets)."""

    def __init__(self, core, metrics=None):
        self.core = core
        self.metrics = metrics

    def _call(self, method: str, msg) -> bytes:
        # through ServingCore.handle so REST traffic shows up in the metrics too
        return self.core.handle("/tensorflow.serving." + method, msg.SerializeToString())

    def _spec(self, msg_spec, name, version, label, sig: Optional[str] = None):
        msg_spec.name = name
        if version is not None:
            msg_spec.version.value = int(version)
        elif label is not None:
            msg_spec.version_label = label
        if sig is not None:
            msg_spec.signature_name = sig

    def _signature(self, name, version, label, sig):
        s = self.core.manager.resolve(name, version, label)
        try:
            return s.signature(sig)
        finally:
            s.release()

    def handle(self, method: str, path: str, body: bytes) -> Tuple[int, str, bytes]:
        """Returns (http status, content type, body)."""
        try:
            if path.rstrip("/") == "/monitoring/prometheus/metrics":
                if method != "GET":
                    raise E.invalid("metrics: use GET")
                text = self.metrics.render() if self.metrics is not None else ""
                return 200, "text/plain; version=0.0.4", text.encode()
            m = _ROUTE.match(path.split("?", 1)[0])
            if m is None:
                raise E.ServingError(E.NOT_FOUND, f"Malformed request: {method} {path}")
            name, version, label, rest = m.group("name"), m.group("version"), m.group("label"), m.group("rest")
            version = int(version) if version is not None else None
            if rest is None or rest == "/metadata":
                if method != "GET":
                    raise E.invalid(f"Malformed request: {method} {path}")
                out = self.status(name, version, label) if rest is None else self.metadata(name, version, label)
            else:
                if method != "POST":
                    raise E.invalid(f"Malformed request: {method} {path}")
                try:
                    req = json.loads(body or b"{}")
                except json.JSONDecodeError as e:
                    raise E.invalid(f"JSON Parse error: {e}") from None
                if not isinstance(req, dict):
                    raise E.invalid("JSON Value: request body must be a JSON object")
                fn = {":predict": self.predict, ":classify": self.classify, ":regress": self.regress}[rest]
                out = fn(name, version, label, req)
            return 200, "application/json", json.dumps(out).encode()
        except E.ServingError as e:
            return HTTP_STATUS.get(e.code, 500), "application/json", json.dumps({"error": e.message}).encode()
        except Exception as e:       # never leak a traceback
            log.exception("REST internal error")
            return 500, "application/json", json.dumps({"error": f"{type(e).__name__}: {e}"}).encode()

    # -------------------------------------------------------------- routes
    def status(self, name, version, label):
        req = serving.GetModelStatusRequest()
        self._spec(req.model_spec, name, version, label)
        resp = serving.GetModelStatusResponse.FromString(self._call("ModelService/GetModelStatus", req))
        return {"model_version_status": [
            {"version": str(s.version), "state": STATE_NAMES.get(s.state, str(s.state)),
             "status": {"error_code": E.CODE_NAMES.get(s.status.error_code, str(s.status.error_code)),
                        "error_message": s.status.error_message}}
            for s in resp.model_version_status]}

    def metadata(self, name, version, label):
        from google.protobuf import json_format
        req = serving.GetModelMetadataRequest()
        self._spec(req.model_spec, name, version, label)
        req.metadata_field.append("signature_def")
        resp = serving.GetModelMetadataResponse.FromString(self._call("PredictionService/GetModelMetadata", req))
        sdm = serving.SignatureDefMap()
        resp.metadata["signature_def"].Unpack(sdm)
        return {"model_spec": {"name": resp.model_spec.name, "signature_name": "",
                               "version": str(resp.model_spec.version.value)},
                "metadata": {"signature_def": json_format.MessageToDict(sdm, preserving_proto_field_name=True)}}

    def predict(self, name, version, label, req: dict):
        sig_req = req.get("signature_name", "")
        sig_name, sigdef = self._signature(name, version, label, sig_req)
        dts = {a: ti.dtype for a, ti in sigdef.inputs.items()}
        row = "instances" in req
        if row == ("inputs" in req):
            raise E.invalid("Missing 'inputs' or 'instances' key" if not row else
                            "Only one of 'inputs' or 'instances' may be specified")
        feeds: Dict[str, np.ndarray] = {}
        if row:
            inst = req["instances"]
            if not isinstance(inst, list) or not inst:
                raise E.invalid("'instances' must be a non-empty JSON list")
            if all(isinstance(x, dict) and set(x) != {"b64"} for x in inst):
                keys = set(inst[0])
                if any(set(x) != keys for x in inst):
                    raise E.invalid("Failed to process element: all instances must have the same named inputs")
                for k in keys:
                    feeds[k] = json_to_array([x[k] for x in inst], dts.get(k, 0))
            else:
                if len(dts) != 1:
                    raise E.invalid("instances without input names require a signature with exactly one input")
                k = next(iter(dts))
                feeds[k] = json_to_array(inst, dts[k])
        else:
            inp = req["inputs"]
            if isinstance(inp, dict) and set(inp) != {"b64"}:
                for k, v in inp.items():
                    feeds[k] = json_to_array(v, dts.get(k, 0))
            else:
                if len(dts) != 1:
                    raise E.invalid("unnamed 'inputs' require a signature with exactly one input")
                k = next(iter(dts))
                feeds[k] = json_to_array(inp, dts[k])
        dtypes = {k: (dts.get(k) or T.dt_of(v)) for k, v in feeds.items()}
        body = native.encode_predict_request(native.spec_tuple(name, version, label, sig_name), feeds,
                                             output_filter=req.get("output_filter", ()), dtypes=dtypes)
        resp = serving.PredictResponse.FromString(self.core.handle("/tensorflow.serving.PredictionService/Predict", body))
        outs = {k: T.tensor_proto_to_numpy(v) for k, v in resp.outputs.items()}
        if not row:
            if len(outs) == 1:
                return {"outputs": array_to_json(next(iter(outs.values())))}
            return {"outputs": {k: array_to_json(v) for k, v in sorted(outs.items())}}
        if len(outs) == 1:
            return {"predictions": array_to_json(next(iter(outs.values())))}
        n = {v.shape[0] if v.ndim else -1 for v in outs.values()}
        if len(n) != 1 or -1 in n:
            raise E.invalid("Tensor name: all output tensors must have the same 0-th dimension size "
                            "for the row format; use the columnar 'inputs' format")
        rows = n.pop()
        return {"predictions": [{k: array_to_json(v[i]) for k, v in sorted(outs.items())} for i in range(rows)]}

    def _input(self, msg_input, req: dict):
        exs = req.get("examples")
        if not isinstance(exs, list) or not exs:
            raise E.invalid("'examples' must be a non-empty JSON list")
        if "context" in req:
            lst = msg_input.example_list_with_context
            lst.context.CopyFrom(example_from_json(req["context"]))
        else:
            lst = msg_input.example_list
        for e in exs:
            lst.examples.add().CopyFrom(example_from_json(e))

    def classify(self, name, version, label, req: dict):
        r = serving.ClassificationRequest()
        self._spec(r.model_spec, name, version, label, req.get("signature_name", ""))
        self._input(r.input, req)
        resp = serving.ClassificationResponse.FromString(self._call("PredictionService/Classify", r))
        return {"result": [[[c.label, c.score] for c in cl.classes] for cl in resp.result.classifications]}

    def regress(self, name, version, label, req: dict):
        r = serving.RegressionRequest()
        self._spec(r.model_spec, name, version, label, req.get("signature_name", ""))
        self._input(r.input, req)
        resp = serving.RegressionResponse.FromString(self._call("PredictionService/Regress", r))
        return {"result": [x.value for x in resp.result.regressions]}


class _Server(ThreadingHTTPServer):
    daemon_threads = True
    allow_reuse_address = True

    def server_bind(self):
        self.socket.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEPORT, 1)
        super().server_bind()


class RestTransport:
    def __init__(self, core, port: int, host: str = "0.0.0.0", metrics=None):
        handler = RestHandler(core, metrics)
        self.handler = handler

        class H(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def _go(self, method):
                n = int(self.headers.get("Content-Length") or 0)
                body = self.rfile.read(n) if n else b""
                code, ctype, out = handler.handle(method, self.path, body)
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(out)))
                self.end_headers()
                self.wfile.write(out)

            def do_GET(self):
                self._go("GET")

            def do_POST(self):
                self._go("POST")

            def log_message(self, fmt, *args):
                log.debug("rest: " + fmt, *args)

        self.httpd = _Server((host, port), H)
        self.port = self.httpd.server_address[1]
        self._thread: Optional[threading.Thread] = None

    def start(self):
        self._thread = threading.Thread(target=self.httpd.serve_forever, name="tfs-rest", daemon=True)
        self._thread.start()
        return self

    def stop(self, grace: Optional[float] = None):
        self.httpd.shutdown()
        self.httpd.server_close()
