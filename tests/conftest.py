import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "distributed-oracle-search_amd")
for p in (PKG, os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (MI355X)")
    config.addinivalue_line("markers", "slow: larger CPU cases")


@pytest.fixture(scope="session")
def root():
    return ROOT


@pytest.fixture(scope="session")
def small_graph():
    import cpd
    return cpd.synth_road_graph(40, 30, seed=7)


@pytest.fixture(scope="session")
def tie_graph():
    """Tiny weights -> many equal-cost paths (multi-bit first-move sets)."""
    import numpy as np
    import cpd
    g = cpd.synth_road_graph(24, 24, seed=11)
    w = (g.w % 3 + 1).astype(np.uint32)
    return cpd.RoadGraph(g.row_ptr, g.dst, w, g.x, g.y)
