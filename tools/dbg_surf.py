import sys; sys.path.insert(0,'.'); sys.path.insert(0,'tests')
import numpy as np
from conftest import scale_rel_err
from fastselect_amd import SURF
from oracle import oracle as O
from sklearn.datasets import make_classification
X, y = make_classification(n_samples=700, n_features=1500, n_informative=20, n_redundant=30, random_state=1)
for star in (False, True):
    g = SURF(backend='gpu', use_star=star).fit(X,y).feature_importances_
    c = SURF(backend='cpu', use_star=star).fit(X,y).feature_importances_
    r = O.surf_scores(X,y,use_star=star)
    print(star, 'gpu-ref', scale_rel_err(g, r), 'cpu-ref', scale_rel_err(c, r), 'gpu-cpu', scale_rel_err(g, c))
