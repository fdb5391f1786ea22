"""The example programs (examples/*.py, mirroring the reference's
examples/*.rs) against a live server on CPU."""
import asyncio
import importlib.util
import os

import numpy as np
import pytest

from rust_tensorflow_serving2_amd.schema import serving
from rust_tensorflow_serving2_amd.server.server import ModelServer, ServerOptions

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, "examples", f"{name}.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


@pytest.fixture(scope="module")
def server(tiny_resnet_path):
    cfg = serving.ModelServerConfig()
    cfg.model_config_list.config.add(name="resnet", base_path=tiny_resnet_path, model_platform="tensorflow")
    srv = ModelServer(ServerOptions(port=0, model_config=cfg, file_system_poll_wait_seconds=0)).start()
    yield srv
    srv.stop()


def test_prediction_example(server, tmp_path):
    from PIL import Image
    img = tmp_path / "example.jpg"
    Image.fromarray(np.random.default_rng(0).integers(0, 256, (32, 32, 3), dtype=np.uint8)).save(img)
    resp = asyncio.run(load("prediction").main([str(img), "-m", "resnet", "--port", str(server.port)]))
    assert set(resp.outputs) == {"classes", "probabilities"}
    assert list(resp.outputs["probabilities"].tensor_shape.dim)[1].size == 11


def test_model_info_example_with_reload(server, tiny_resnet_path):
    status, md = asyncio.run(load("model_info").main(
        ["-m", "resnet", "--port", str(server.port), "--reload-base-path", tiny_resnet_path]))
    assert status.model_version_status[0].state == 30
    assert md.model_spec.name == "resnet"
    assert [n for n, _v, _s in server.manager.available()] == ["resnet"]     # still serving


def test_async_example(server):
    res = asyncio.run(load("async_requests").main(["-m", "resnet", "--port", str(server.port)]))
    assert len(res) == 2 and not any(isinstance(r, BaseException) for r in res)


def test_make_models(tmp_path):
    import subprocess
    import sys
    r = subprocess.run([sys.executable, os.path.join(ROOT, "serving", "make_models.py"), "--root", str(tmp_path),
                        "--models", "half_plus_two"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "half_plus_two" / "1" / "saved_model.pb").exists()
    assert (tmp_path / "example.jpg").exists()
