import sys, os, json, numpy as np
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from dpgo_amd import hip as H
from oracle import dpgo_oracle as O
k = int(sys.argv[1])
g = H.Graph.grid3d(k, seed=0)
r, d, b = 5, 3, 4
YL = H.lifting_matrix(3, r)
X, it, rr = g.chordal_init_gpu(r, YL, rtol=1e-10, max_iters=50000)
P = O.to_poses(X, r, d)
Y = P[:, :, :d]
G = np.einsum('nra,nrb->nab', Y, Y) - np.eye(d)
err = np.abs(G).reshape(len(Y), -1).max(axis=1)
Q = O.qf(Y)
qerr = np.abs(Q - Y).reshape(len(Y), -1).max(axis=1)
print(json.dumps({"iters": it, "relres": rr, "orth_max": float(err.max()), "worst_pose": int(err.argmax()),
                  "qf_minus_Y_max": float(qerr.max()), "n_qf_bad": int((qerr > 1e-8).sum()),
                  "bad_examples": [int(i) for i in np.nonzero(qerr > 1e-8)[0][:10]]}))
i = int(qerr.argmax())
print(Y[i]); print(Q[i])
