"""Shared test set-up.

Markers: `gpu` = needs a real MI355X (runs through the HIP C-ABI); everything else runs on the
CPU (oracle pins, scene ingest, ABI surface, gloo multi-process logic).
"""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "project3-cuda-path-tracer-2025_amd")
ORACLE = os.path.join(REPO, "oracle")
SCENES = os.path.join(REPO, "scenes")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (PKG, ORACLE):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")


def scene_path(name):
    return os.path.join(SCENES, name if name.endswith(".json") else name + ".json")


@pytest.fixture(scope="session")
def oracle():
    import oracle as O
    return O


@pytest.fixture(scope="session")
def ptamd():
    import ptamd as P
    return P
