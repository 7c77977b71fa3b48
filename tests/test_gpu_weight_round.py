"""dbsr_weights_round_diffuse (error-diffusion rounding of the DBSR convs' weights to fp16 / bf16, the engine's
default: DBSREngine.WEIGHT_ROUNDING) against a numpy restatement of the same carried rounding -- bitwise: every
step is one fp32 subtraction, one round-to-nearest-even conversion and one fp32 addition -- plus its contract: every
value representable in the dtype, within one ulp (of the channel's largest weight) of the fp32 weight, each output
channel's error sum within half such an ulp."""
import numpy as np
import pytest
import torch

DEV = 'cuda'
pytestmark = pytest.mark.gpu


def _round16(x, dt):
    x = np.float32(x)
    if dt == torch.float16:
        return np.float32(np.float16(x))
    u = np.array([x], dtype=np.float32).view(np.uint32)[0]
    u = (u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000            # round to nearest even (finite values)
    return np.array([u], dtype=np.uint32).view(np.float32)[0]


def _diffuse_np(w, dt):
    co, ci, kh, kw = w.shape
    f = w.transpose(0, 2, 3, 1).reshape(co, -1)                  # K order: tap-major, then input channel
    q = np.empty_like(f)
    for o in range(co):
        e = np.float32(0)
        for k in range(f.shape[1]):
            v = f[o, k]
            t = _round16(np.float32(v - e), dt)
            e = np.float32(e + np.float32(t - v))
            q[o, k] = t
    return q.reshape(co, kh, kw, ci).transpose(0, 3, 1, 2)


@pytest.mark.parametrize('shape,dt', [((16, 64, 3, 3), torch.float16), ((8, 96, 3, 3), torch.bfloat16),
                                      ((32, 64, 1, 1), torch.float16), ((4, 565, 3, 3), torch.float16)])
def test_weights_round_diffuse(shape, dt):
    from dbsr_amd import _lib as L
    gen = torch.Generator().manual_seed(sum(shape))
    w = torch.randn(*shape, generator=gen) * (2.0 / (shape[1] * shape[2] * shape[3])) ** 0.5
    wd = w.to(DEV)
    out = torch.empty_like(wd)
    L.check(L.lib().dbsr_weights_round_diffuse(wd.data_ptr(), shape[0], shape[1], shape[2], shape[3],
                                               L.dtype_code(dt), out.data_ptr(), torch.cuda.current_stream().cuda_stream),
            'dbsr_weights_round_diffuse')
    torch.cuda.synchronize()
    q = out.cpu()
    ref = torch.from_numpy(_diffuse_np(w.numpy(), dt))
    assert torch.equal(q, ref)
    assert torch.equal(q.to(dt).float(), q)                      # representable: the pack keeps it
    ulp = (w.abs().clamp_min(2 ** -14) * (2.0 ** -10 if dt == torch.float16 else 2.0 ** -7))   # >= the true ulp
    umax = ulp.reshape(shape[0], -1).max(dim=1).values
    # each weight within one ulp of its channel's largest weight (the carried error is at most half of one)
    assert bool(((q - w).abs().reshape(shape[0], -1) <= umax[:, None] * (1 + 1e-6)).all())
    err = (q - w).reshape(shape[0], -1).sum(dim=1).abs()
    assert bool((err <= 0.5 * umax * (1 + 1e-3)).all()), err.max()
    # against round-to-nearest: the per-channel error sums are much smaller
    near = (w.to(dt).float() - w).reshape(shape[0], -1).sum(dim=1).abs()
    assert err.mean() < near.mean()


def test_weights_round_diffuse_rejects():
    from dbsr_amd import _lib as L
    lib = L.lib()
    assert lib.dbsr_weights_round_diffuse(None, 4, 4, 3, 3, L.DBSR_F16, None, None) == -1
    x = torch.zeros(4, device=DEV)
    assert lib.dbsr_weights_round_diffuse(x.data_ptr(), 1, 4, 1, 1, L.DBSR_F32, x.data_ptr() + 64, None) == -1
    assert lib.dbsr_weights_round_diffuse(x.data_ptr(), 1, 2048, 3, 3, L.DBSR_F16, x.data_ptr() + 64, None) == -1
