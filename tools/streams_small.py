import sys; sys.path.insert(0, '.')
import torch, bench, latticeum_amd as LA
from latticeum_amd import dist as LD
for S in (4, 6, 8, 4):
    r = bench.extra_shape(LA, torch, LD, None, 0, 0, 1, 1024, 464, 32, S, 384, 24, 'small')
    print(S, round(r['value'], 1), flush=True)
