"""First-run vs steady-state equality of the bf16 forward (same net, same input, eager runs)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import dbsr_amd
from dbsr_amd import _lib
if os.environ.get('CHK_ALGO'):
    _lib.lib().dbsr_set_conv_algo(int(os.environ['CHK_ALGO']))
from dbsr_amd.burst import synthetic_bursts

B, N, H, W = [int(v) for v in (sys.argv[1:5] if len(sys.argv) > 4 else (8, 14, 48, 48))]
dt = torch.float32 if len(sys.argv) > 5 and sys.argv[5] == 'fp32' else torch.bfloat16
burst, _ = synthetic_bursts(B, N, H, W, sr_factor=8, seed=9)
burst = burst.cuda()
net = dbsr_amd.build_synthetic_net(seed=0).cuda().eval()
net.set_compute_dtype(dt)
outs = []
with torch.no_grad():
    for _ in range(3):
        pred, aux = net(burst)
        outs.append((pred.clone(), aux['offsets'].clone()))
for i in (1, 2):
    print(sys.argv[1:], {k: v for k, v in os.environ.items() if k.startswith(('DBSR_', 'CHK_'))}, 'run', i,
          'offsets maxdiff vs run0 %.3g' % (outs[i][1] - outs[0][1]).abs().max().item(),
          'vs run1 %.3g' % (outs[i][1] - outs[1][1]).abs().max().item(),
          'pred maxdiff vs run0 %.3g' % (outs[i][0] - outs[0][0]).abs().max().item())
