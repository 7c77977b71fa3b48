"""Per-conv cycle stamps of dbsr_pwc_extract (diagnostic stamp build) at the bench shape (112 frames of 64x64).
Build: make exp EXP_FLAGS=-DDBSR_EXT_STAMPS EXP_NAME=extst
Run:   DBSR_HIP_LIB=deep-rawburst-sr_amd/libdbsr_hip_extst.so python tools/ext_stamps.py"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dbsr_amd import _lib as L                                   # noqa: E402
from dbsr_amd.engine import NHWC, PWC_LEVEL_CH, PackedConv, cpad   # noqa: E402


def main():
    dev = torch.device('cuda')
    dt = torch.float16
    s = torch.cuda.current_stream().cuda_stream
    fn = L.lib().dbsr_diag_ext_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_longlong]
    F = 112
    rgb = NHWC(F, 64, 64, 8, dt, dev)
    rgb.t[..., :3].uniform_()
    convs = (L.PwcExtConv * 18)()
    lv = (L.Tensor * 6)()
    keep, levels = [], []
    hw = 64
    for k in range(6):
        C, Cin = PWC_LEVEL_CH[k + 1], (3 if k == 0 else PWC_LEVEL_CH[k])
        hw //= 2
        levels.append(NHWC(F, hw, hw, cpad(C), dt, dev))
        lv[k] = levels[-1].d(0)
        for j in range(3):
            ci = Cin if j == 0 else C
            pc = PackedConv(torch.nn.Conv2d(ci, C, 3, stride=2 if j == 0 else 1, padding=1).to(dev), dt, dev, s)
            keep.append(pc)
            convs[3 * k + j] = L.PwcExtConv(pc.w.data_ptr(), pc.bias.data_ptr(), ci, C, 2 if j == 0 else 1)
    for rep in range(3):
        fn(None, 0)
        L.check(L.lib().dbsr_pwc_extract(F, 64, 64, rgb.d(0), convs, lv, s), 'extract')
        torch.cuda.synchronize()
    buf = np.zeros(128 * 8 * 40, dtype=np.uint64)
    fn(buf.ctypes.data, buf.size)
    st = buf.reshape(128, 8, 40)[:F].astype(np.int64)
    t0 = st[:, :, 0].min(axis=1, keepdims=True)
    rel = (st - t0[:, :, None]).astype(np.float64)
    med = np.median(rel.max(axis=1), axis=0)          # per block: the last wave to reach each stamp
    mean = rel.mean(axis=1)                            # per block: the average wave
    for ci in range(18):
        a_, b_ = 1 + 2 * ci, 2 + 2 * ci
        nxt = 3 + 2 * ci if ci < 17 else 39
        print('L%d.c%d  compute: last wave %7.0f (mean wave %7.0f)  barrier wait %7.0f' % (
            ci // 3 + 1, ci % 3, np.median(rel[:, :, b_].max(axis=1) - rel[:, :, a_].max(axis=1)),
            np.median(mean[:, b_] - mean[:, a_]), np.median(rel[:, :, nxt].max(axis=1) - rel[:, :, b_].max(axis=1))))
    print('total %.0f s_memtime ticks' % np.median(rel[:, :, 39].max(axis=1)))


if __name__ == '__main__':
    main()
