"""dbsr_amd — MI355X-native (gfx950) DBSR forward path.

Drop-in for the reference's hot path (Tony-Tseng/deep-rawburst-sr, models/dbsr + models/alignment +
external/pwcnet): hand-written HIP kernels in libdbsr_hip.so behind a C ABI (include/dbsr_hip.h),
driven from the module API the reference's callers use (`net(burst) -> (pred, aux)`).
"""
from .dbsrnet import DBSRNet, dbsrnet_cvpr2021, build_synthetic_net, DBSR_SYNTHETIC_KWARGS  # noqa: F401
from .pwcnet import PWCNet  # noqa: F401
