"""Async client with the reference's API surface (``src/lib.rs``), in Python.

=====================================  =========================================
reference (Rust)                       here
=====================================  =========================================
``TensorflowServing::new()`` builder   ``TensorflowServing.new()`` ->
  ``.hostname() .port()                ``TensorflowServingBuilder`` with the same
  .signature_name() .build().await``   setters and ``await .build()``
  (src/lib.rs:72-146)                  (same error strings, same default
                                       ``"serving_default"``)
``impl Clone`` (src/lib.rs:148-156)    ``clone()`` (shares the HTTP/2 channel)
``classify`` (src/lib.rs:176-202)      ``classify`` — returns the result (the
                                       reference panics after the RPC)
``predict_with_preprocessing``         same (image -> ``[1, W, H, 3]`` f32
  (src/lib.rs:204-267)                 ``float_val`` under alias ``"input"``)
``predict`` (src/lib.rs:269-282)       same
``model_status`` / ``model_metadata``  same
  / ``reload`` (src/lib.rs:284-334)
dead ``regress`` / ``multi_inference`` implemented
  (src/lib.rs:336-410)
``ModelDescription`` / ``Payload`` /   ``ModelDescription`` / ``Payload`` /
  ``Image`` (src/lib.rs:13-43,450-572) ``to_image``
``pub use ModelConfig`` (:70)          ``ModelConfig``
=====================================  =========================================

Request bodies are encoded by the native codec (packed float arrays are a
single memcpy), and responses are upb message objects.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Callable, Dict, Iterable, List, Mapping, Optional, Sequence, Union

import numpy as np

from .. import native
from ..schema import MODEL_SERVICE, PREDICTION_SERVICE, ModelConfig, serving, tf  # noqa: F401
from ..utils import tensors as T

__all__ = ["TensorflowServing", "TensorflowServingBuilder", "ModelDescription", "Payload",
           "ModelConfig", "TFServingError", "to_image"]

MAX_MESSAGE = 2 ** 31 - 1


class TFServingError(Exception):
    """A failed RPC or client-side error (``Box<dyn Error>`` in the reference)."""

    def __init__(self, message: str, code=None):
        super().__init__(message)
        self.code = code
        self.message = message


@dataclass
class ModelDescription:
    """``ModelDescription<S>{name, version: Option<i64>}`` (src/lib.rs:450-482)."""
    name: str
    version: Optional[int] = None

    @classmethod
    def of(cls, m: Union["ModelDescription", str]) -> "ModelDescription":
        if isinstance(m, ModelDescription):
            return m
        if isinstance(m, (str, bytes)):
            return cls(m.decode() if isinstance(m, bytes) else m)
        raise TypeError(f"cannot build a ModelDescription from {type(m).__name__}")


class Payload:
    """``Payload::{Bytes, Ints, Floats}`` (src/lib.rs:484-538)."""

    def __init__(self, kind: str, values):
        if kind not in ("bytes", "ints", "floats"):
            raise ValueError(kind)
        self.kind = kind
        self.values = list(values)

    @classmethod
    def bytes(cls, values: Iterable[bytes]) -> "Payload":
        return cls("bytes", values)

    @classmethod
    def ints(cls, values: Iterable[int]) -> "Payload":
        return cls("ints", values)

    @classmethod
    def floats(cls, values: Iterable[float]) -> "Payload":
        return cls("floats", values)

    @classmethod
    def of(cls, v) -> "Payload":
        if isinstance(v, Payload):
            return v
        vals = list(v) if not isinstance(v, (bytes, str, int, float)) else [v]
        if all(isinstance(x, (bytes, bytearray, str)) for x in vals):
            return cls.bytes([x.encode() if isinstance(x, str) else bytes(x) for x in vals])
        if all(isinstance(x, (int, np.integer)) and not isinstance(x, bool) for x in vals):
            return cls.ints(vals)
        return cls.floats([float(x) for x in vals])

    def to_feature(self) -> "tf.Feature":
        f = tf.Feature()
        if self.kind == "bytes":
            f.bytes_list.value.extend(self.values)
        elif self.kind == "ints":
            f.int64_list.value.extend(int(x) for x in self.values)
        else:
            f.float_list.value.extend(float(x) for x in self.values)
        return f


def to_image(img):
    """``Image::to_image`` (src/lib.rs:13-43): path / str / PathLike / PIL image / HxWxC uint8 array."""
    from PIL import Image
    if isinstance(img, Image.Image):
        return img.copy()
    if isinstance(img, (str, os.PathLike)):
        return Image.open(img)
    if isinstance(img, np.ndarray):
        return Image.fromarray(img)
    raise TypeError(f"cannot convert {type(img).__name__} to an image")


def _preprocess_lut(preprocessing_fn: Callable) -> np.ndarray:
    """``preprocessing_fn`` at the 256 values a u8 pixel can take (as f32, the
    way src/lib.rs:237-242 feeds it): the whole per-pixel map as a table."""
    vals = np.arange(256, dtype=np.float32)
    try:
        out = np.asarray(preprocessing_fn(vals), dtype=np.float32)
        if out.shape != vals.shape:
            raise ValueError
    except Exception:
        out = np.array([preprocessing_fn(float(v)) for v in vals], dtype=np.float32)
    return np.ascontiguousarray(out)


def _image_request(spec, img, preprocessing_fn: Callable, alias: str = "input") -> bytes:
    """The reference's predict_with_preprocessing request (src/lib.rs:226-263)
    built natively: u8 pixels -> table lookup -> packed float_val, one pass."""
    im = to_image(img)
    w, h = im.size
    px = np.ascontiguousarray(np.asarray(im, dtype=np.uint8)).reshape(-1)
    return native.encode_image_request(spec, alias, px, [1, w, h, 3], _preprocess_lut(preprocessing_fn))


def _image_tensor(img, preprocessing_fn: Callable) -> np.ndarray:
    """Pixels exactly as the reference builds them: dims ``[1, width, height, 3]``
    (src/lib.rs:229-235 — width/height in that order) over ``raw_pixels()`` in
    row-major H x W x native-channels order, each mapped through
    ``preprocessing_fn`` (vectorised when the function allows it)."""
    im = to_image(img)
    w, h = im.size
    px = np.asarray(im, dtype=np.uint8).astype(np.float32).reshape(-1)
    try:
        out = np.asarray(preprocessing_fn(px), dtype=np.float32)
        if out.shape != px.shape:
            raise ValueError
    except Exception:
        out = np.fromiter((preprocessing_fn(float(p)) for p in px), dtype=np.float32, count=px.size)
    return out, [1, w, h, 3]


def _status_code(e):
    try:
        return e.code()
    except Exception:
        return None


class TensorflowServingBuilder:
    """``TensorflowServingBuilder`` (src/lib.rs:86-146)."""

    def __init__(self):
        self._hostname: Optional[str] = None
        self._port: Optional[int] = None
        self._signature_name: Optional[str] = None
        self._options: list = []

    def hostname(self, hostname: str) -> "TensorflowServingBuilder":
        self._hostname = str(hostname)
        return self

    def port(self, port: int) -> "TensorflowServingBuilder":
        if not (0 <= int(port) <= 65535):
            raise ValueError("port must fit in u16")
        self._port = int(port)
        return self

    def signature_name(self, signature_name: str) -> "TensorflowServingBuilder":
        self._signature_name = str(signature_name)
        return self

    def channel_options(self, options: list) -> "TensorflowServingBuilder":
        self._options = list(options)
        return self

    async def build(self) -> "TensorflowServing":
        import grpc
        if self._hostname is None:
            raise TFServingError("hostname not provided")
        if self._port is None:
            raise TFServingError("port not provided")
        sig = self._signature_name if self._signature_name is not None else "serving_default"
        self._signature_name = None   # `.take()` semantics
        opts = [("grpc.max_receive_message_length", MAX_MESSAGE),
                ("grpc.max_send_message_length", MAX_MESSAGE)] + self._options
        channel = grpc.aio.insecure_channel(f"{self._hostname}:{self._port}", options=opts)
        try:
            await channel.channel_ready()
        except Exception as e:
            await channel.close()
            raise TFServingError(f"transport error: {e}") from None
        return TensorflowServing(channel, sig)


class TensorflowServing:
    """The client (src/lib.rs:161-334).  Safe for concurrent use; ``clone()``
    shares the underlying HTTP/2 connection (examples/async.rs pattern)."""

    def __init__(self, channel, signature_name: str):
        self._channel = channel
        self.signature_name_ = signature_name
        self._calls = {}

    @staticmethod
    def new() -> TensorflowServingBuilder:
        return TensorflowServingBuilder()

    def clone(self) -> "TensorflowServing":
        c = TensorflowServing(self._channel, self.signature_name_)
        return c

    __copy__ = clone

    async def close(self):
        await self._channel.close()

    async def __aenter__(self):
        return self

    async def __aexit__(self, *exc):
        await self.close()

    # ------------------------------------------------------------ plumbing
    async def _call(self, service: str, method: str, request: bytes, resp_cls, timeout=None):
        import grpc
        path = f"/{service}/{method}"
        stub = self._calls.get(path)
        if stub is None:
            stub = self._channel.unary_unary(path)
            self._calls[path] = stub
        try:
            raw = await stub(request, timeout=timeout)
        except grpc.aio.AioRpcError as e:
            raise TFServingError(f"status: {e.code().name}, message: {e.details()!r}", _status_code(e)) from None
        return raw if resp_cls is None else resp_cls.FromString(raw)

    def _model_spec(self, model) -> "serving.ModelSpec":
        """``build_model_spec`` (src/lib.rs:433-447): version as Int64Value; label never set."""
        md = ModelDescription.of(model)
        ms = serving.ModelSpec(name=md.name, signature_name=self.signature_name_)
        if md.version is not None:
            ms.version.value = int(md.version)
        return ms

    def _spec_tuple(self, model):
        md = ModelDescription.of(model)
        return native.spec_tuple(md.name, md.version, None, self.signature_name_)

    @staticmethod
    def _input(payload_map: Mapping[str, object]) -> "serving.Input":
        """``build_input`` (src/lib.rs:412-431): one Example in an ExampleList."""
        inp = serving.Input()
        ex = inp.example_list.examples.add()
        for k, v in payload_map.items():
            ex.features.feature[str(k)].CopyFrom(Payload.of(v).to_feature())
        return inp

    # ------------------------------------------------------------ API
    async def classify(self, model, payload_map: Mapping[str, object], timeout=None):
        req = serving.ClassificationRequest()
        req.model_spec.CopyFrom(self._model_spec(model))
        req.input.CopyFrom(self._input(payload_map))
        resp = await self._call(PREDICTION_SERVICE, "Classify", req.SerializeToString(),
                                serving.ClassificationResponse, timeout)
        return resp.result

    async def regress(self, model, payload_map: Mapping[str, object], timeout=None):
        req = serving.RegressionRequest()
        req.model_spec.CopyFrom(self._model_spec(model))
        req.input.CopyFrom(self._input(payload_map))
        resp = await self._call(PREDICTION_SERVICE, "Regress", req.SerializeToString(),
                                serving.RegressionResponse, timeout)
        return resp.result

    async def multi_inference(self, model, tasks: Sequence[tuple], payload_map: Mapping[str, object],
                              timeout=None):
        """tasks: [(signature_name, method_name)] all on ``model``."""
        md = ModelDescription.of(model)
        req = serving.MultiInferenceRequest()
        for sig, method in tasks:
            t = req.tasks.add(method_name=method)
            t.model_spec.name = md.name
            t.model_spec.signature_name = sig
            if md.version is not None:
                t.model_spec.version.value = md.version
        req.input.CopyFrom(self._input(payload_map))
        return await self._call(PREDICTION_SERVICE, "MultiInference", req.SerializeToString(),
                                serving.MultiInferenceResponse, timeout)

    async def predict_with_preprocessing(self, img, model_description, preprocessing_fn: Callable,
                                         timeout=None):
        # shape [1, w, h, 3] from the image, float_val = fn(pixel) for every raw
        # pixel (reference quirks preserved), encoded by the native image encoder
        body = _image_request(self._spec_tuple(model_description), img, preprocessing_fn)
        return await self._call(PREDICTION_SERVICE, "Predict", body, serving.PredictResponse, timeout)

    async def predict(self, img, model_description, timeout=None):
        return await self.predict_with_preprocessing(img, model_description, lambda p: p, timeout)

    async def predict_tensors(self, model, inputs: Mapping[str, np.ndarray], output_filter: Sequence[str] = (),
                              timeout=None, raw: bool = False):
        """Extension: arbitrary named tensors in, ``{alias: ndarray}`` out."""
        body = native.encode_predict_request(self._spec_tuple(model), dict(inputs), output_filter)
        raw_resp = await self._call(PREDICTION_SERVICE, "Predict", body, None, timeout)
        if raw:
            return raw_resp
        resp = serving.PredictResponse.FromString(raw_resp)
        return {k: T.tensor_proto_to_numpy(v) for k, v in resp.outputs.items()}

    async def model_status(self, model, timeout=None):
        req = serving.GetModelStatusRequest()
        req.model_spec.CopyFrom(self._model_spec(model))
        return await self._call(MODEL_SERVICE, "GetModelStatus", req.SerializeToString(),
                                serving.GetModelStatusResponse, timeout)

    async def model_metadata(self, model, timeout=None):
        req = serving.GetModelMetadataRequest(metadata_field=["signature_def"])
        req.model_spec.CopyFrom(self._model_spec(model))
        return await self._call(PREDICTION_SERVICE, "GetModelMetadata", req.SerializeToString(),
                                serving.GetModelMetadataResponse, timeout)

    async def reload(self, model_config: Union[Sequence["serving.ModelConfig"], "serving.ModelConfig"],
                     timeout=None):
        if isinstance(model_config, serving.ModelConfig):
            model_config = [model_config]
        req = serving.ReloadConfigRequest()
        for mc in model_config:
            req.config.model_config_list.config.add().CopyFrom(mc)
        return await self._call(MODEL_SERVICE, "HandleReloadConfigRequest", req.SerializeToString(),
                                serving.ReloadConfigResponse, timeout)


def _encode_float_request(spec, alias: str, values: np.ndarray, dims: List[int]) -> bytes:
    """PredictRequest with one DT_FLOAT ``float_val`` tensor whose shape is
    ``dims`` regardless of len(values) (the reference may send mismatching
    counts, e.g. RGBA images — the server must reject, not crash)."""
    from ..schema import serving as S
    if int(np.prod(dims)) == values.size:
        return native.encode_predict_request(spec, {alias: values.reshape(dims)})
    # the count disagrees with the shape: encode the values, then patch the shape
    body = native.encode_predict_request(spec, {alias: values.reshape(-1)})
    req = S.PredictRequest.FromString(body)
    t = req.inputs[alias]
    del t.tensor_shape.dim[:]
    for d in dims:
        t.tensor_shape.dim.add(size=d)
    return req.SerializeToString()


def unpack_signature_defs(metadata_response) -> Dict[str, "tf.SignatureDef"]:
    """Helper: ``GetModelMetadataResponse.metadata["signature_def"]`` -> {name: SignatureDef}."""
    sdm = serving.SignatureDefMap()
    metadata_response.metadata["signature_def"].Unpack(sdm)
    return dict(sdm.signature_def)
