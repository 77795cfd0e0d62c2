import sys, time
sys.path.insert(0, 'repic-copy_amd'); sys.path.insert(0, '.')
import numpy as np
from scipy.sparse import coo_matrix
from scipy.optimize import linprog
from oracle import cpu_vec
from repic_amd import synth
cfg = synth.SynthConfig(**synth.CONFIGS["C5"], seed=0)
mg = synth.batch(cfg, 1)[0]
xs, ys, ss = (np.concatenate([t[j] for t in mg]) for j in range(3))
t0 = time.time()
o = cpu_vec.micrograph(xs, ys, ss, [len(t[0]) for t in mg], cfg.box)
C = len(o["w"]); V = o["V"]
print("cliques", C, "V", V, "oracle s", time.time() - t0, flush=True)
rows = o["rows"].reshape(-1)
A = coo_matrix((np.ones(len(rows)), (rows, np.repeat(np.arange(C), cfg.k))), shape=(V, C)).tocsr()
w = np.asarray(o["w"], np.float64)
t0 = time.time()
r = linprog(-w, A_ub=A, b_ub=np.ones(V), bounds=(0, 1), method="highs")
print("LP", r.status, -r.fun, "s", time.time() - t0, flush=True)
x = r.x
print("fractional", int(((x > 1e-6) & (x < 1 - 1e-6)).sum()), "ones", int((x > 1 - 1e-6).sum()))
np.save("/tmp/c5_lp_x.npy", x)
