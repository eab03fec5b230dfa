import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
# the benchmarks' scene modules (kitti_scenes, tum_rgbd_scenes, match_scenes) feed the tests too
sys.path.insert(0, str(ROOT / "benchmarks"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through liborbx.so on the GPU)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.build()
    return O


@pytest.fixture(scope="session")
def orbx_built():
    from orbslam2commentedbyxcm_amd import build
    build.build()
    return build.LIB
