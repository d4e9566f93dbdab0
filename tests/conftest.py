"""Shared test setup.

Markers: ``gpu`` = needs an MI355X (run on the GPU box with ``-m gpu``).
The oracle (``oracle/``) is imported here only as the checker.
"""
import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "lance-distributed-training_amd")
for p in (PKG, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run with -m gpu")


def has_gpu() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if has_gpu():
        return
    skip = pytest.mark.skip(reason="no HIP device in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def sampler_golden():
    with open(os.path.join(GOLDEN, "sampler.json")) as f:
        return json.load(f)


def read_golden(rel: str) -> bytes:
    with open(os.path.join(GOLDEN, rel), "rb") as f:
        return f.read()
