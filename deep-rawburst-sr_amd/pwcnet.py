"""PWC-Net alignment network (models/alignment/pwcnet.py:234-281), MI355X engine-backed.

`PWCNet(source_img, target_img) -> flow[P,2,H,W]` is the reference's own sub-seam
(pwcnet.py:248); it runs the HIP PWC path of engine.py.  The reference loads
`pwcnet-network-default.pth` with `strKey.replace('module', 'net')` (pwcnet.py:244-246); same here.
"""
import torch
import torch.nn as nn

from .arch import PWCNetwork


class PWCNet(nn.Module):
    def __init__(self, load_pretrained=True, weights_path=None, rgb2bgr=False):
        super().__init__()
        self.net = PWCNetwork()
        self.rgb2bgr = rgb2bgr
        if load_pretrained:
            if weights_path is None:
                raise ValueError('load_pretrained=True needs weights_path (pwcnet.py:240-242)')
            weights_dict = torch.load(weights_path, map_location='cpu', weights_only=True)
            self.net.load_state_dict({k.replace('module', 'net'): v for k, v in weights_dict.items()})
        self.compute_dtype = torch.float32
        self._engine = None

    def forward(self, source_img, target_img):
        if source_img.shape[-2:] != target_img.shape[-2:]:
            raise ValueError('source/target spatial sizes differ (pwcnet.py:249-250)')
        from .engine import PWCEngine
        if self._engine is None or not self._engine.matches(self):
            self._engine = PWCEngine(self)
        return self._engine.forward(source_img, target_img)
