"""Drop-in DBSR network for MI355X.

Mirrors the reference's module API:
  DBSRNet(encoder, merging, decoder).forward(im[B,N,4,H,W]) -> (pred[B,3,sH,sW],
      {'offsets': [B,N-1,2,H,W], 'fusion_weights': [B,N,C,H,W]})        models/dbsr/dbsrnet.py:24-38
  dbsrnet_cvpr2021(...)  (same signature and defaults)                    models/dbsr/dbsrnet.py:41-82
with identical state_dict keys, so a reference checkpoint loads with `load_state_dict` and
admin/loading.load_network(..., constructor_module='dbsr_amd.dbsrnet') rebuilds this class
(admin/loading.py:72-75).

The forward never runs torch compute kernels: it hands device pointers to the HIP engine
(engine.py -> libdbsr_hip.so).  There is no CPU fallback: a CPU tensor or a missing library raises.
"""
import torch
import torch.nn as nn

from . import arch
from .pwcnet import PWCNet


class ResEncoderWarpAlignnet(nn.Module):
    """Parameter holder for models/dbsr/encoders.py:21-46."""
    def __init__(self, init_dim, num_res_blocks, out_dim, alignment_net, activation='relu',
                 train_alignmentnet=True, warp_type='bilinear'):
        super().__init__()
        if warp_type != 'bilinear':
            raise NotImplementedError('only bilinear warp is on the hot path (encoders.py:80)')
        self.warp_type = warp_type
        self.alignment_net = alignment_net
        self.train_alignmentnet = train_alignmentnet
        self.init_layer = arch.conv_block(4, init_dim, 3, padding=1, activation=activation)
        self.res_layers = nn.Sequential(*[arch.ResBlock(init_dim, init_dim, activation=activation)
                                          for _ in range(num_res_blocks)])
        self.out_layer = arch.conv_block(init_dim, out_dim, 3, padding=1, activation=activation)


class WeightedSum(nn.Module):
    """Parameter holder for models/dbsr/merging.py:21-59."""
    def __init__(self, input_dim, project_dim, offset_feat_dim, num_offset_feat_extractor_res=1,
                 num_weight_predictor_res=1, use_offset=True, offset_modulo=None, ref_offset_noise=0.0,
                 softmax=True, use_base_frame=False, activation='relu'):
        super().__init__()
        self.use_offset = use_offset
        self.offset_modulo = offset_modulo
        self.ref_offset_noise = ref_offset_noise
        self.softmax = softmax
        self.use_base_frame = use_base_frame
        self.feat_project_layer = arch.conv_block(input_dim, project_dim, 1, padding=0, activation=activation)
        ofe = [arch.conv_block(2, offset_feat_dim, 3, padding=1, activation=activation)]
        ofe += [arch.ResBlock(offset_feat_dim, offset_feat_dim, activation=activation)
                for _ in range(num_offset_feat_extractor_res)]
        self.offset_feat_extractor = nn.Sequential(*ofe)
        wp = [arch.conv_block(project_dim * 2 + offset_feat_dim * use_offset, 2 * project_dim, 3, padding=1,
                              activation=activation)]
        wp += [arch.ResBlock(2 * project_dim, 2 * project_dim, activation=activation)
               for _ in range(num_weight_predictor_res)]
        wp.append(arch.conv_block(2 * project_dim, input_dim, 3, padding=1, activation='none'))
        self.weight_predictor = nn.Sequential(*wp)


class ResPixShuffleConv(nn.Module):
    """Parameter holder for models/dbsr/decoders.py:20-52."""
    def __init__(self, input_dim, init_conv_dim, num_pre_res_blocks, post_conv_dim, num_post_res_blocks,
                 activation='relu', upsample_factor=2, icnrinit=False, gauss_blur_sd=None, gauss_ksz=3):
        super().__init__()
        self.gauss_ksz = gauss_ksz
        self.init_layer = arch.conv_block(input_dim, init_conv_dim, 3, padding=1, activation=activation)
        self.pre_res_layers = nn.Sequential(*[arch.ResBlock(init_conv_dim, init_conv_dim, activation=activation)
                                              for _ in range(num_pre_res_blocks)])
        self.upsample_layer = arch.PixShuffleUpsampler(init_conv_dim, post_conv_dim, upsample_factor=upsample_factor,
                                                       activation=activation, icnrinit=icnrinit,
                                                       gauss_blur_sd=gauss_blur_sd, gauss_ksz=gauss_ksz)
        self.post_res_layers = nn.Sequential(*[arch.ResBlock(post_conv_dim, post_conv_dim, activation=activation)
                                               for _ in range(num_post_res_blocks)])
        self.predictor = arch.conv_block(post_conv_dim, 3, 1, padding=0)


class DBSRNet(nn.Module):
    """Deep Burst Super-Resolution model (models/dbsr/dbsrnet.py:24-38).

    Extra knobs (not in the reference; defaults keep reference behaviour):
      compute_dtype      torch.float32 (default, parity mode), torch.bfloat16 (throughput mode) or
                         torch.float16 (configs[4]);
                         accumulation is fp32 in both, flows/offsets stay fp32.
      return_fusion_weights  True: aux['fusion_weights'] is produced exactly as the reference
                         returns it (shape [B,N,C,H,W]; backed by the engine's channels-last buffer).
      use_graph          capture the forward into a HIP graph per input shape and replay it.  Outputs
                         are fresh tensors (cloned from the graph's static buffers) like the reference's.
      graph_zero_copy    with use_graph: return views of the static buffers instead (no clone); they are
                         overwritten by the next forward of the same shape.
      zero_flow          configs[0]'s identity-flow alignment stub (offsets = 0, no PWC-Net); changing it
                         rebuilds the engine.
    In training mode with autograd enabled (net.train(), no torch.no_grad()) the forward keeps its
    activations and `pred` carries a grad_fn: loss.backward() on any objective fills the DBSR parameters'
    .grad (PWC-Net is frozen, encoders.py:56-61) from the HIP backward kernels, and any torch.optim optimizer
    steps them (compute dtype float32 or bfloat16).  Evaluation (net.eval() or no_grad) runs the inference
    engine.
    """
    def __init__(self, encoder, merging, decoder):
        super().__init__()
        self.encoder = encoder
        self.merging = merging
        self.decoder = decoder
        self.compute_dtype = torch.float32
        self.return_fusion_weights = True
        self.use_graph = False
        self.zero_flow = False          # config 1's identity-flow alignment stub
        self.graph_zero_copy = False
        self._engine = None
        self._train_engine = None

    def set_compute_dtype(self, dtype):
        if dtype not in (torch.float32, torch.bfloat16, torch.float16):
            raise ValueError('compute_dtype must be torch.float32, torch.bfloat16 or torch.float16')
        self.compute_dtype = dtype
        self._engine = None
        self._train_engine = None
        return self

    def _get_engine(self):
        from .engine import DBSREngine
        if self._engine is None or not self._engine.matches(self):
            self._engine = DBSREngine(self)
        return self._engine

    def _trains(self):
        """Training mode with autograd on: some DBSR (non-PWC) parameter requires grad."""
        if not (self.training and torch.is_grad_enabled()):
            return False
        return any(p.requires_grad for n, p in self.named_parameters() if not n.startswith('encoder.alignment_net'))

    def forward(self, im):
        if im.dim() != 5:
            raise ValueError('expected burst [B,N,4,H,W], got shape {}'.format(tuple(im.shape)))
        if self._trains():
            # autograd through the HIP training forward / backward (training.train_forward): the reference's
            # loop -- pred, _ = net(burst); loss.backward(); optimizer.step() -- runs unchanged
            from .training import train_forward
            return train_forward(self, im)
        return self._get_engine().forward(im)


def dbsrnet_cvpr2021(enc_init_dim, enc_num_res_blocks, enc_out_dim,
                     dec_init_conv_dim, dec_num_pre_res_blocks, dec_post_conv_dim, dec_num_post_res_blocks,
                     upsample_factor=2, activation='relu', train_alignmentnet=False,
                     offset_feat_dim=64, weight_pred_proj_dim=32, num_offset_feat_extractor_res=1,
                     num_weight_predictor_res=1, offset_modulo=1.0, use_offset=True, ref_offset_noise=0.0,
                     softmax=True, use_base_frame=True, icnrinit=False, gauss_blur_sd=None, gauss_ksz=3,
                     pwcnet_weights_path=None):
    """models/dbsr/dbsrnet.py:41-82.  `pwcnet_weights_path`: optional PWC-Net checkpoint (the
    reference reads it from env_settings().pretrained_nets_dir); None leaves PWC weights to a later
    load_state_dict of a full DBSR checkpoint, which carries them under encoder.alignment_net.*."""
    if activation != 'relu':
        raise NotImplementedError('only relu activation is on the hot path')
    # softmax, use_base_frame and offset_modulo take any value the reference accepts (the engine's variants,
    # engine.merging_variant); use_offset=False and ref_offset_noise > 0 are refused there and here
    if not use_offset or ref_offset_noise > 0.0:
        raise NotImplementedError('hot path needs use_offset=True and ref_offset_noise=0 (merging.py:91-96)')
    alignment_net = PWCNet(load_pretrained=pwcnet_weights_path is not None, weights_path=pwcnet_weights_path)
    encoder = ResEncoderWarpAlignnet(enc_init_dim, enc_num_res_blocks, enc_out_dim, alignment_net,
                                     activation=activation, train_alignmentnet=train_alignmentnet)
    merging = WeightedSum(enc_out_dim, weight_pred_proj_dim, offset_feat_dim,
                          num_offset_feat_extractor_res=num_offset_feat_extractor_res,
                          num_weight_predictor_res=num_weight_predictor_res, offset_modulo=offset_modulo,
                          use_offset=use_offset, ref_offset_noise=ref_offset_noise, softmax=softmax,
                          use_base_frame=use_base_frame)
    decoder = ResPixShuffleConv(enc_out_dim, dec_init_conv_dim, dec_num_pre_res_blocks, dec_post_conv_dim,
                                dec_num_post_res_blocks, upsample_factor=upsample_factor, activation=activation,
                                gauss_blur_sd=gauss_blur_sd, icnrinit=icnrinit, gauss_ksz=gauss_ksz)
    net = DBSRNet(encoder=encoder, merging=merging, decoder=decoder)
    net.arch_kwargs = dict(enc_init_dim=enc_init_dim, enc_num_res_blocks=enc_num_res_blocks,
                           enc_out_dim=enc_out_dim, dec_init_conv_dim=dec_init_conv_dim,
                           dec_num_pre_res_blocks=dec_num_pre_res_blocks, dec_post_conv_dim=dec_post_conv_dim,
                           dec_num_post_res_blocks=dec_num_post_res_blocks, upsample_factor=upsample_factor,
                           offset_feat_dim=offset_feat_dim, weight_pred_proj_dim=weight_pred_proj_dim,
                           num_offset_feat_extractor_res=num_offset_feat_extractor_res,
                           num_weight_predictor_res=num_weight_predictor_res, icnrinit=icnrinit,
                           gauss_blur_sd=gauss_blur_sd, gauss_ksz=gauss_ksz)
    return net


DBSR_SYNTHETIC_KWARGS = dict(   # train_settings/dbsr/default_synthetic.py:73-82 (downsample_factor=4)
    enc_init_dim=64, enc_num_res_blocks=9, enc_out_dim=512,
    dec_init_conv_dim=64, dec_num_pre_res_blocks=5,
    dec_post_conv_dim=32, dec_num_post_res_blocks=4,
    upsample_factor=8, offset_feat_dim=64, weight_pred_proj_dim=64,
    num_weight_predictor_res=3, gauss_blur_sd=1.0, icnrinit=True)


def build_synthetic_net(seed=0, kwargs=None):
    """dbsrnet_cvpr2021 with the default_synthetic architecture and seeded weights (weights.py)."""
    from .weights import generate_state_dict
    net = dbsrnet_cvpr2021(**(kwargs or DBSR_SYNTHETIC_KWARGS))
    sd = generate_state_dict(arch.state_dict_shapes(net), seed=seed)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    return net
