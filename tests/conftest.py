import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "maveric-slam_amd")
for p in (os.path.join(ROOT, "oracle"), PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")


def load_golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.fixture(scope="session")
def golden():
    return load_golden


@pytest.fixture(scope="session")
def orc():
    import oracle

    oracle.lib()
    return oracle


@pytest.fixture(scope="session")
def ctx():
    import mvtrack

    if mvtrack.device_count() <= 0:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    c = mvtrack.Context(0)
    yield c
    c.close()


@pytest.fixture(params=["i8", "i8s", "f16"])
def screen(request, ctx):
    """every fp32 screen (int8 MFMA one-pass -- the default --, int8 against a staged image, fp16
    MFMA) must give identical outputs"""
    ctx.set_allpairs_screen(request.param)
    yield request.param
    ctx.set_allpairs_screen("i8")


@pytest.fixture(scope="session")
def torch_cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("torch sees no GPU")
    return torch


@pytest.fixture(scope="session")
def image0(golden):
    d = golden("quantized_image0.npz")
    return dict(rows=int(d["feature_rows"]), cols=int(d["feature_cols"]), semi=d["semi"], desc=d["desc"],
                semi_scale=np.float32(d["semi_scale"]), desc_scale=np.float32(d["desc_scale"]))
