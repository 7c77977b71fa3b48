"""Per-stage timeline of the pipelined conv kernel from the stamps build
(make exp EXP_NAME=stamps EXP_FLAGS=-DDBSR_PIPE_STAMPS).
Usage: DBSR_HIP_LIB=.../libdbsr_hip_stamps.so python tools/pipe_stamps.py <shape-substring>"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dbsr_amd import _lib as L                      # noqa: E402
from dbsr_amd.engine import NHWC, PackedConv, Plan, cpad  # noqa: E402
from tools.bench_conv import SHAPES                 # noqa: E402


def main():
    sub = sys.argv[1]
    name, F, H, W, cin, cout, k = [s for s in SHAPES if sub in s[0]][0]
    dev = torch.device('cuda')
    dt = torch.bfloat16
    st = torch.cuda.current_stream().cuda_stream
    conv = torch.nn.Conv2d(cin, cout, k, padding=k // 2).to(dev)
    pc = PackedConv(conv, dt, dev, st)
    x = NHWC(F, H, W, cpad(cin), dt, dev)
    x.t.normal_()
    y = NHWC(F, H, W, max(8, (cout + 7) // 8 * 8), dt, dev)
    r = NHWC(F, H, W, max(8, (cout + 7) // 8 * 8), dt, dev)
    plan = Plan()
    plan.conv(name, pc, F, x, 0, (H, W), y, 0, L.ACT_NONE, res=r, post_act=L.ACT_RELU)
    plan.finalize_workspace(dev)
    lib = L.lib()
    lib.dbsr_debug_pipe_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.lib().dbsr_set_conv_algo(3)
    for _ in range(5):
        plan.run(st)
    torch.cuda.synchronize()
    lib.dbsr_debug_pipe_stamps_clear()
    plan.run(st)
    torch.cuda.synchronize()
    buf = np.zeros(256 * 128, dtype=np.uint64)
    lib.dbsr_debug_pipe_stamps(buf.ctypes.data, buf.size)
    st_ = buf.reshape(256, 128).astype(np.int64)
    t0 = st_[:, 0][st_[:, 0] > 0].min()
    print(f'{name}: block start spread {(st_[:, 0].max() - t0)} cyc')
    for b in [0, 1, 7, 100, 255]:
        row = st_[b]
        n = int(np.nonzero(row)[0].max()) + 1
        rel = row[:n] - row[0]
        segs = []
        for s in range((n - 2) // 4):
            a = row[1 + 4 * s:5 + 4 * s]
            segs.append('s%d bar %d iss %d cmp %d' % (s, a[1] - a[0], a[2] - a[1], a[3] - a[2]))
        print(f'block {b}: start +{row[0] - t0} total {rel[-1]}  ' + ' | '.join(segs))
    tot = [(r[np.nonzero(r)[0].max()] - r[0]) for r in st_ if r[0] > 0]
    print('block totals (cyc): min %d median %d max %d' % (min(tot), int(np.median(tot)), max(tot)))


if __name__ == '__main__':
    main()
