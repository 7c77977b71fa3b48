"""Conv wgrad microbenchmark at the training step's shapes (configs[3], bf16): per-launch device time of
dbsr_conv_wgrad_bias for the LDS-DMA ring kernel (algo 1) and the register-staged kernel (algo 0), queued
behind a spin kernel so the host stays ahead.  Usage: python tools/bench_wgrad.py [--only name] [--algos 1,0]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dbsr_amd  # noqa: F401,E402
from dbsr_amd import _lib as L  # noqa: E402

SHAPES = {                      # name: (frames, h, w, cin, cout, k)
    'wp.res': (104, 128, 128, 128, 128, 3),
    'enc.res': (112, 128, 128, 64, 64, 3),
    'wp.out': (104, 128, 128, 128, 512, 3),
    'dec.post': (8, 1024, 1024, 32, 32, 3),
    'proj.oth': (104, 128, 128, 512, 64, 1),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--only', default=None)
    ap.add_argument('--algos', default='1,0')
    ap.add_argument('--reps', type=int, default=10)
    args = ap.parse_args()
    dev = torch.device('cuda')
    lib = L.lib()
    s = torch.cuda.current_stream().cuda_stream
    for name, (n, h, w, ci, co, k) in SHAPES.items():
        if args.only and args.only not in name:
            continue
        ldx, ldy = (ci + 31) // 32 * 32, (co + 31) // 32 * 32
        x = torch.randn(n, h, w, ldx, device=dev).to(torch.bfloat16)
        dy = torch.randn(n, h, w, ldy, device=dev).to(torch.bfloat16)
        dw = torch.zeros(co * ci * k * k, device=dev)
        db = torch.zeros(co, device=dev)
        need = lib.dbsr_conv_wgrad_workspace_bytes(n, h, w, ci, co, k)
        ws = torch.empty(need // 4 + 1, device=dev)
        flop = 2.0 * n * h * w * ci * co * k * k
        for a in [int(v) for v in args.algos.split(',')]:
            L.check(lib.dbsr_set_wgrad_algo(a), 'algo')
            call = lambda: L.check(lib.dbsr_conv_wgrad_bias(n, h, w, L.tensor_desc(x, ldx), ci, L.tensor_desc(dy, ldy), co, k,  # noqa: E731
                                                            dw.data_ptr(), db.data_ptr(), 0, ws.data_ptr(), need, s), 'wgrad')
            call()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda._sleep(2_000_000)
            e0.record()
            for _ in range(args.reps):
                call()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / args.reps
            print('%-9s algo %d  %8.1f us  %6.1f TF/s  (%.3f of 2.5 PF)' % (name, a, us, flop / us / 1e6, flop / us / 1e6 / 2500))
        L.lib().dbsr_set_wgrad_algo(1)
        del x, dy


if __name__ == '__main__':
    main()
