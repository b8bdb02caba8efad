"""Debug probe: resnet_tiny under bf16 autocast, fused BN path vs stock
modules -- relative difference of every conv input and of the logits."""
import copy
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from distributed_kfac_pytorch_amd.models import resnet  # noqa: E402
from distributed_kfac_pytorch_amd.ops import bn as fbn  # noqa: E402

DEV = 'cuda'
torch.manual_seed(0)
m1 = resnet.resnet_tiny(num_classes=10).to(DEV).to(memory_format=torch.channels_last)
m2 = copy.deepcopy(m1)
x = torch.randn(8, 3, 64, 64, device=DEV).to(memory_format=torch.channels_last)
caps = []
for m in (m1, m2):
    d = {}
    for name, mod in m.named_modules():
        if isinstance(mod, (nn.Conv2d, nn.Linear)):
            mod.register_forward_pre_hook(lambda mod, inp, name=name, d=d: d.__setitem__(
                name, (inp[0].detach().float().clone(), inp[0].stride(), inp[0].dtype)))
    caps.append(d)
outs = []
for m, fused in ((m1, True), (m2, False)):
    fbn.ENABLED = fused
    with torch.autocast('cuda', dtype=torch.bfloat16):
        outs.append(m(x).float())
fbn.ENABLED = True
for name in caps[0]:
    a, sa, da = caps[0][name]
    b, sb, db = caps[1][name]
    r = ((a - b).norm() / max(b.norm().item(), 1e-30)).item()
    print('%-28s rel %.2e  %s %s  %s %s' % (name, r, da, sa, db, sb))
print('logits rel', ((outs[0] - outs[1]).norm() / outs[1].norm()).item())
