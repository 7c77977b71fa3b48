"""Microbenchmark of dbsr_conv2d on the cfg2 hot shapes: kernel selections (dbsr_set_conv_algo) side by side, fp16.
Usage: python tools/bench_conv.py"""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dbsr_amd import _lib as L                     # noqa: E402
from dbsr_amd.engine import NHWC, PackedConv, Plan, cpad  # noqa: E402

SHAPES = [  # name, frames, H, W, cin, cout, k
    ('enc.res 64->64', 112, 48, 48, 64, 64, 3),
    ('enc.c1 64->64', 112, 48, 48, 64, 64, 3),
    ('enc.out 64->512', 112, 48, 48, 64, 512, 3),
    ('wp.init 192->128', 112, 48, 48, 192, 128, 3),
    ('wp.res 128->128', 112, 48, 48, 128, 128, 3),
    ('wp.res 128->128 (104 frames)', 104, 48, 48, 128, 128, 3),
    ('wp.c1 128->128 (104 frames)', 104, 48, 48, 128, 128, 3),
    ('wp.out 128->512', 112, 48, 48, 128, 512, 3),
    ('dec.post 32->32', 8, 384, 384, 32, 32, 3),
    ('dec.pre 64->64', 8, 48, 48, 64, 64, 3),
    ('dec.init 512->64', 8, 48, 48, 512, 64, 3),
    ('enc.init 4->64', 112, 48, 48, 4, 64, 3),
    ('ofe.init 2->64', 112, 48, 48, 2, 64, 3),
    ('proj 512->64 1x1', 104, 48, 48, 512, 64, 1),
    ('pwc.dec2.d4 544->32', 104, 16, 16, 544, 32, 3),
    ('pwc.dec2.flow 576->2', 104, 16, 16, 565, 2, 3),
    ('pwc.dec4.d3 480->64', 104, 4, 4, 469, 64, 3),
    ('pwc.dec6.d4 544->32', 104, 1, 1, 529, 32, 3),
]


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument('--only', default=None, help='substring of the shape names to run')
    ap.add_argument('--algos', default='2,1,0')
    ap.add_argument('--reps', type=int, default=20)
    args = ap.parse_args()
    algos = [int(a) for a in args.algos.split(',')]
    dev = torch.device('cuda')
    dt = torch.float16
    s = torch.cuda.current_stream().cuda_stream
    for name, F, H, W, cin, cout, k in SHAPES:
        if args.only and args.only not in name:
            continue
        conv = torch.nn.Conv2d(cin, cout, k, padding=k // 2).to(dev)
        pc = PackedConv(conv, dt, dev, s)
        x = NHWC(F, H, W, cpad(cin), dt, dev)
        x.t.normal_()
        y = NHWC(F, H, W, max(8, (cout + 7) // 8 * 8), dt, dev)
        plan = Plan()
        if 'res' in name or 'post' in name or 'pre' in name:
            r = NHWC(F, H, W, max(8, (cout + 7) // 8 * 8), dt, dev)
            plan.conv(name, pc, F, x, 0, (H, W), y, 0, L.ACT_NONE, res=r, post_act=L.ACT_RELU)
        else:
            plan.conv(name, pc, F, x, 0, (H, W), y, 0, L.ACT_RELU)
        flop = plan.work[0][1]
        plan.finalize_workspace(dev)
        out = []
        for algo in algos:
            L.lib().dbsr_set_conv_algo(algo)
            ms = plan.time_ops(s, reps=args.reps)[0][1]
            out.append('%s %7.1f us %6.1f TF/s' % (['generic', 'tiled', 'auto', 'pipe', 'no-ws', 'ws8'][algo], ms * 1e3, flop / ms / 1e9))
        L.lib().dbsr_set_conv_algo(2)
        print(f'{name:22s} ' + ' | '.join(out))


if __name__ == '__main__':
    main()
