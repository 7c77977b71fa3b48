import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, 'tests', 'golden')


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (HIP) device and the built libdbsr_hip.so')


@pytest.fixture(scope='session')
def golden():
    import numpy as np

    def load(name):
        return dict(np.load(os.path.join(GOLDEN, name + '.npz'), allow_pickle=False))
    return load


@pytest.fixture(scope='session')
def synth_sd():
    """Seeded synthetic weights (seed 0) for the default_synthetic architecture, as torch CPU fp32."""
    import torch
    import dbsr_amd
    from dbsr_amd import arch
    from dbsr_amd.weights import generate_state_dict
    net = dbsr_amd.dbsrnet_cvpr2021(**dbsr_amd.DBSR_SYNTHETIC_KWARGS)
    sd = generate_state_dict(arch.state_dict_shapes(net), seed=0)
    return {k: torch.from_numpy(v) for k, v in sd.items()}
