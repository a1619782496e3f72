"""Generates tests/golden/goku_kmeans_z300.npy: the Goku inducing points of the reference's
SingleBin / latent SVGP notebooks, KMeans(n_clusters=300, random_state=42).fit(X_train)
.cluster_centers_ (notebooks/demo: goku power spectra.ipynb cell 10; its printed rows are the
goku_kmeans_z300_rows KAT).  X_train = the Goku training inputs (normalised, fidelity column),
restated by oracle/mfgp_oracle.load_powerspecs.  sklearn 1.7.2; run from the repo root."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from sklearn.cluster import KMeans  # noqa: E402

from oracle.mfgp_oracle import load_powerspecs  # noqa: E402

d = load_powerspecs(os.path.join(ROOT, "tests", "golden", "data",
                                 "matter_power_1128_Box1000_Part750_36_Box1000_Part3000_z0"))
Z = KMeans(n_clusters=300, random_state=42).fit(d["X"]).cluster_centers_
np.save(os.path.join(ROOT, "tests", "golden", "goku_kmeans_z300.npy"), Z)
print(Z.shape, "fractional-fidelity rows:", int(np.sum((Z[:, -1] != 0) & (Z[:, -1] != 1))))
