"""Parameter tree of the DBSR network, with the reference's exact state_dict keys.

These nn.Module classes only HOLD parameters (so `load_state_dict` of a reference checkpoint works
unchanged, admin/loading.py:87); they never run torch compute.  The forward path is the HIP engine
(engine.py).  Names follow:
  conv_block / ResBlock            models/layers/blocks.py:46-96
  PixShuffleUpsampler              models/layers/upsampling.py:22-49
  ResEncoderWarpAlignnet           models/dbsr/encoders.py:21-46
  WeightedSum                      models/dbsr/merging.py:21-59
  ResPixShuffleConv                models/dbsr/decoders.py:20-52
  PWC-Net Network / PWCNet         models/alignment/pwcnet.py:41-246
"""
from collections import OrderedDict

import torch.nn as nn


def conv_block(in_planes, out_planes, kernel_size=3, stride=1, padding=1, dilation=1, bias=True,
               activation='relu'):
    layers = [nn.Conv2d(in_planes, out_planes, kernel_size=kernel_size, stride=stride, padding=padding,
                        dilation=dilation, bias=bias)]
    if activation == 'relu':
        layers.append(nn.ReLU(inplace=True))
    elif activation != 'none':
        raise ValueError('Unknown activation {}'.format(activation))
    return nn.Sequential(*layers)


class ResBlock(nn.Module):
    def __init__(self, inplanes, planes, activation='relu'):
        super().__init__()
        self.conv1 = conv_block(inplanes, planes, 3, padding=1, activation=activation)
        self.conv2 = conv_block(planes, planes, 3, padding=1, activation='none')


class PixShuffleUpsampler(nn.Module):
    def __init__(self, input_dim, output_dim, upsample_factor=2, activation='relu', icnrinit=False,
                 gauss_blur_sd=None, gauss_ksz=3):
        super().__init__()
        self.conv_layer = conv_block(input_dim, output_dim * upsample_factor ** 2, 1, padding=0,
                                     activation=activation, bias=not icnrinit)
        self.upsample_factor = upsample_factor
        self.gauss_blur_sd = gauss_blur_sd
        self.gauss_ksz = gauss_ksz


def _lrelu():
    return nn.LeakyReLU(negative_slope=0.1)


class PWCExtractor(nn.Module):
    def __init__(self):
        super().__init__()
        chans = [3, 16, 32, 64, 96, 128, 196]
        for i, name in enumerate(['netOne', 'netTwo', 'netThr', 'netFou', 'netFiv', 'netSix']):
            ci, co = chans[i], chans[i + 1]
            setattr(self, name, nn.Sequential(
                nn.Conv2d(ci, co, 3, 2, 1), _lrelu(), nn.Conv2d(co, co, 3, 1, 1), _lrelu(),
                nn.Conv2d(co, co, 3, 1, 1), _lrelu()))


PWC_CURRENT = {2: 81 + 32 + 2 + 2, 3: 81 + 64 + 2 + 2, 4: 81 + 96 + 2 + 2, 5: 81 + 128 + 2 + 2, 6: 81}
PWC_DENSE_OUT = [128, 128, 96, 64, 32]


class PWCDecoder(nn.Module):
    def __init__(self, level):
        super().__init__()
        cur = PWC_CURRENT[level]
        if level < 6:
            prev = PWC_CURRENT[level + 1]
            self.netUpflow = nn.ConvTranspose2d(2, 2, 4, 2, 1)
            self.netUpfeat = nn.ConvTranspose2d(prev + 128 + 128 + 96 + 64 + 32, 2, 4, 2, 1)
        cin = cur
        for name, co in zip(['netOne', 'netTwo', 'netThr', 'netFou', 'netFiv'], PWC_DENSE_OUT):
            setattr(self, name, nn.Sequential(nn.Conv2d(cin, co, 3, 1, 1), _lrelu()))
            cin += co
        self.netSix = nn.Sequential(nn.Conv2d(cin, 2, 3, 1, 1))


class PWCRefiner(nn.Module):
    def __init__(self):
        super().__init__()
        chans = [81 + 32 + 2 + 2 + 128 + 128 + 96 + 64 + 32, 128, 128, 128, 96, 64, 32, 2]
        dil = [1, 2, 4, 8, 16, 1, 1]
        layers = []
        for i, d in enumerate(dil):
            layers.append(nn.Conv2d(chans[i], chans[i + 1], 3, 1, d, dilation=d))
            if i < 6:
                layers.append(_lrelu())
        self.netMain = nn.Sequential(*layers)


class PWCNetwork(nn.Module):
    def __init__(self):
        super().__init__()
        self.netExtractor = PWCExtractor()
        self.netTwo = PWCDecoder(2)
        self.netThr = PWCDecoder(3)
        self.netFou = PWCDecoder(4)
        self.netFiv = PWCDecoder(5)
        self.netSix = PWCDecoder(6)
        self.netRefiner = PWCRefiner()


def state_dict_shapes(module):
    return OrderedDict((k, tuple(v.shape)) for k, v in module.state_dict().items())
