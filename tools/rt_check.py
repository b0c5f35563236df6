import os, sys
sys.path.insert(0, '.')
import fastselect_amd
from fastselect_amd import _lib
import torch
print('torch', torch.__version__, 'cuda avail', torch.cuda.is_available(), torch.cuda.device_count())
print('fs devices', _lib.device_count())
maps = open('/proc/self/maps').read()
libs = sorted(set(l.split()[-1] for l in maps.splitlines() if 'amdhip64' in l or 'hsa-runtime' in l))
print('\n'.join(libs))
import numpy as np
from sklearn.datasets import make_classification
X, y = make_classification(n_samples=300, n_features=200, random_state=0)
s = fastselect_amd.MultiSURF(backend='gpu').fit(X, y).feature_importances_
t = torch.ones(4, device='cuda')
print('ok', s[:3], t.sum().item())
