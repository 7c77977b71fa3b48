"""Per-conv cycle stamps of dbsr_pwc_dense at each coarse PWC level (diagnostic stamp build).
Build: make exp EXP_FLAGS=-DDBSR_PIPE_STAMPS EXP_NAME=stamps
Run:   DBSR_HIP_LIB=deep-rawburst-sr_amd/libdbsr_hip_stamps.so python tools/dense_stamps.py"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dbsr_amd import _lib as L                                   # noqa: E402
from dbsr_amd.engine import BASE_OFF, DENSE_OFF, DENSE_OUT, NHWC, PWC_LEVEL_CH, PackedConv, cpad   # noqa: E402


def main():
    dev = torch.device('cuda')
    dt = torch.bfloat16
    s = torch.cuda.current_stream().cuda_stream
    fn = L.lib().dbsr_diag_dense_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_longlong]
    P = 104
    for level, hw in ((6, 1), (5, 2), (4, 4), (3, 8)):
        C = PWC_LEVEL_CH[level]
        base_real = 81 if level == 6 else 81 + C + 4
        ld = BASE_OFF + cpad(base_real)
        D = NHWC(P, hw, hw, ld, dt, dev)
        D.t.normal_()
        fl = NHWC(P, hw, hw, 8, torch.float32, dev)
        convs = (L.PwcDenseConv * 6)()
        cin = base_real
        keep = []
        for i in range(6):
            cout = DENSE_OUT[i] if i < 5 else 2
            pc = PackedConv(torch.nn.Conv2d(cin, cout, 3, padding=1).to(dev), dt, dev, s)
            keep.append(pc)
            cg = cpad(cin) // 8
            start = 0 if i == 5 else (BASE_OFF if i == 0 else DENSE_OFF[i - 1])
            convs[i] = L.PwcDenseConv(pc.w.data_ptr(), pc.bias.data_ptr(), 9 * cg * 8, cg, start, cout,
                                      DENSE_OFF[i] if i < 5 else 0)
            if i < 5:
                cin += DENSE_OUT[i]
        for _ in range(5):
            L.check(L.lib().dbsr_pwc_dense(P, hw, hw, D.d(0), BASE_OFF, convs, fl.d(0), s), 'dense')
        torch.cuda.synchronize()
        fn(None, 0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        L.check(L.lib().dbsr_pwc_dense(P, hw, hw, D.d(0), BASE_OFF, convs, fl.d(0), s), 'dense')
        e1.record()
        torch.cuda.synchronize()
        buf = np.zeros(128 * 8 * 16, dtype=np.uint64)
        fn(buf.ctypes.data, buf.size)
        st = buf.reshape(128, 8, 16).astype(np.int64)
        live = st[:, :, 0] > 0
        nb = int(live.any(axis=1).sum())
        print(f'level {level} ({hw}x{hw}): {e0.elapsed_time(e1) * 1e3:.1f} us, {nb} blocks')
        w0 = st[:, 0][live[:, 0]]
        tot = np.median(w0[:, 13] - w0[:, 0])
        print('  wave0 median: tile load %.0f' % np.median(w0[:, 1] - w0[:, 0]),
              ' '.join('conv%d %.0f/%.0f' % (c, np.median(w0[:, 2 + 2 * c] - w0[:, 1 + 2 * c]),
                                             np.median((w0[:, 3 + 2 * c] if c < 5 else w0[:, 13]) - w0[:, 1 + 2 * c]))
                       for c in range(6)), 'total %.0f' % tot)


if __name__ == '__main__':
    main()
