import sys, time, numpy as np
sys.path.insert(0, '.')
from ldbc_graphalytics_platforms_graphblas_amd import algorithms as A
from ldbc_graphalytics_platforms_graphblas_amd.graphio import rmat
from oracle import oracle as O
scale = int(sys.argv[1])
ctx = A.Context(0)
csr = rmat(scale, 16, 3, undirected=True)
G = A.Graph(ctx, csr, False)
t = time.time()
got = A.LA_PR(G, 0.85, 10)
print('scale', scale, 'done in', time.time() - t, 'max rel err', float(np.max(np.abs(got - O.pagerank(csr, False, 0.85, 10)) / O.pagerank(csr, False, 0.85, 10))), flush=True)
G.close(); ctx.close()
