"""SavedModel directory I/O.

Layout (the one TF Serving and the reference's fixture use,
``serving/fetch.sh:22-26``)::

    <base_path>/<version>/saved_model.pb          SavedModel{meta_graphs}
    <base_path>/<version>/variables/variables.index / .data-00000-of-00001
    <base_path>/<version>/assets/...

``load`` picks the MetaGraphDef whose tags match (default ``{"serve"}``) and
returns its graph, signatures and a lazily-verified TensorBundle.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional

import numpy as np

from ..schema import tf
from .bundle import Bundle, DataLossError, write_bundle

SAVED_MODEL_FILENAME_PB = "saved_model.pb"
VARIABLES_DIR = "variables"
VARIABLES_PREFIX = "variables"
DEFAULT_TAGS = ("serve",)


class SavedModelError(IOError):
    pass


@dataclass
class SavedModelBundle:
    export_dir: str
    meta_graph: "tf.MetaGraphDef"
    bundle: Optional[Bundle]
    tags: List[str] = field(default_factory=list)

    @property
    def graph_def(self):
        return self.meta_graph.graph_def

    @property
    def signatures(self) -> Dict[str, "tf.SignatureDef"]:
        return dict(self.meta_graph.signature_def)


def write_saved_model(export_dir: str, graph_def, signatures: Dict[str, "tf.SignatureDef"],
                      variables: Optional[Dict[str, np.ndarray]] = None,
                      var_dtypes: Optional[Dict[str, int]] = None,
                      saver_def=None, tags: Iterable[str] = DEFAULT_TAGS,
                      assets: Optional[Dict[str, bytes]] = None) -> str:
    os.makedirs(export_dir, exist_ok=True)
    sm = tf.SavedModel(saved_model_schema_version=1)
    mg = sm.meta_graphs.add()
    mg.meta_info_def.tags.extend(tags)
    mg.meta_info_def.meta_graph_version = "v1"
    mg.meta_info_def.tensorflow_version = "rust_tensorflow_serving2_amd"
    mg.graph_def.CopyFrom(graph_def)
    if saver_def is not None:
        mg.saver_def.CopyFrom(saver_def)
    for k, v in signatures.items():
        mg.signature_def[k].CopyFrom(v)
    if variables:
        write_bundle(os.path.join(export_dir, VARIABLES_DIR, VARIABLES_PREFIX), variables, var_dtypes)
    else:
        os.makedirs(os.path.join(export_dir, VARIABLES_DIR), exist_ok=True)
    if assets:
        adir = os.path.join(export_dir, "assets")
        os.makedirs(adir, exist_ok=True)
        for name, data in assets.items():
            with open(os.path.join(adir, name), "wb") as f:
                f.write(data)
    tmp = os.path.join(export_dir, SAVED_MODEL_FILENAME_PB + ".tmp")
    with open(tmp, "wb") as f:
        f.write(sm.SerializeToString())
    os.replace(tmp, os.path.join(export_dir, SAVED_MODEL_FILENAME_PB))
    return export_dir


def maybe_saved_model_directory(export_dir: str) -> bool:
    return os.path.isfile(os.path.join(export_dir, SAVED_MODEL_FILENAME_PB))


def load(export_dir: str, tags: Iterable[str] = DEFAULT_TAGS, verify: bool = True) -> SavedModelBundle:
    pb_path = os.path.join(export_dir, SAVED_MODEL_FILENAME_PB)
    if not os.path.isfile(pb_path):
        if os.path.isfile(os.path.join(export_dir, "saved_model.pbtxt")):
            from google.protobuf import text_format
            with open(os.path.join(export_dir, "saved_model.pbtxt")) as f:
                sm = text_format.Parse(f.read(), tf.SavedModel())
        else:
            raise SavedModelError(f"no SavedModel found at {export_dir}")
    else:
        with open(pb_path, "rb") as f:
            data = f.read()
        try:
            sm = tf.SavedModel.FromString(data)
        except Exception as e:  # upb DecodeError
            raise DataLossError(f"{pb_path}: cannot parse SavedModel: {e}") from None
    want = set(tags)
    chosen = None
    for mg in sm.meta_graphs:
        if set(mg.meta_info_def.tags) == want:
            chosen = mg
            break
    if chosen is None:
        avail = [list(mg.meta_info_def.tags) for mg in sm.meta_graphs]
        raise SavedModelError(f"{export_dir}: no MetaGraphDef with tags {sorted(want)} (have {avail})")
    prefix = os.path.join(export_dir, VARIABLES_DIR, VARIABLES_PREFIX)
    bundle = Bundle(prefix, verify=verify) if os.path.isfile(prefix + ".index") else None
    return SavedModelBundle(export_dir, chosen, bundle, list(chosen.meta_info_def.tags))
