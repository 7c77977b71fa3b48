"""Deterministic synthetic weights for the DBSR state_dict.

No pretrained weights exist offline (install.sh:88-96 downloads them), so parity and
benchmarks run on seeded weights.  Every tensor is drawn from its own numpy PCG64 stream keyed by
(seed, crc32(state_dict key)), so the result does not depend on key order, on torch's RNG, or on
the machine: the GPU box regenerates byte-identical weights without the reference.

Distribution: U(-g/sqrt(fan_in), +g/sqrt(fan_in)) with torch's fan_in rule (tensor.size(1) * kernel
area, also for ConvTranspose2d).  g = sqrt(3) keeps activation variance roughly constant through a
linear layer (torch's default init uses g = 1, under which a 40-conv random network decays to ~0 and
makes parity checks vacuous).  At this gain the random PWC-Net produces flows of ~1-2 px on the
synthetic bursts, so the warps exercise sub-pixel and border cases.
"""
import math
import zlib
from collections import OrderedDict

import numpy as np

DEFAULT_GAIN = math.sqrt(3.0)


def _fan_in(shape):
    if len(shape) < 2:
        return None
    rf = 1
    for s in shape[2:]:
        rf *= s
    return shape[1] * rf


def generate_state_dict(shapes, seed=0, gain=DEFAULT_GAIN):
    """shapes: OrderedDict key -> tuple shape (from the module tree).  Returns OrderedDict of float32
    numpy arrays."""
    out = OrderedDict()
    weight_fan = {}
    for k, shp in shapes.items():
        if k.endswith('.weight'):
            weight_fan[k[:-len('.weight')]] = _fan_in(shp)
    for k, shp in shapes.items():
        stem = k.rsplit('.', 1)[0]
        fan = weight_fan.get(stem) or _fan_in(shp) or 1
        bound = gain / math.sqrt(fan)
        rng = np.random.Generator(np.random.PCG64([int(seed), zlib.crc32(k.encode())]))
        out[k] = rng.uniform(-bound, bound, size=shp).astype(np.float32)
    return out
