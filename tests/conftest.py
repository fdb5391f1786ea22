import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

REFERENCE = "/root/reference"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")
    config.addinivalue_line("markers", "slow: long-running test")
    # native CPU extension is required by nearly everything: build it once
    from rust_tensorflow_serving2_amd import _build
    _build.build_cpu()


@pytest.fixture(scope="session")
def models_dir(tmp_path_factory):
    return tmp_path_factory.mktemp("models")


@pytest.fixture(scope="session")
def hpt_path(models_dir):
    from rust_tensorflow_serving2_amd.models import half_plus_two
    base = os.path.join(str(models_dir), "half_plus_two")
    half_plus_two.export(os.path.join(base, "1"))
    return base


@pytest.fixture(scope="session")
def tiny_resnet_path(models_dir):
    """A narrow, shallow ResNet (same graph vocabulary) that runs fast on CPU."""
    from rust_tensorflow_serving2_amd.models import resnet
    base = os.path.join(str(models_dir), "tiny_resnet")
    resnet.export(os.path.join(base, "1"), blocks=(1, 1, 1, 1), width=8, num_classes=11,
                  image_size=32, seed=1)
    return base


def reference_available():
    return os.path.isdir(os.path.join(REFERENCE, "protos"))
