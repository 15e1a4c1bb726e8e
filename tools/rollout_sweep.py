import sys; sys.path.insert(0, "tools")
from sweep_step import run, load_network
n28, n199, tt = load_network("bittner28"), load_network("bittner199"), load_network("tt200")
for rep in range(2):
    run(n28, 65536, 1, 1, rollout=256, sb=256)
    run(n199, 65536, 1, 1, rollout=256, sb=256)
    run(n199, 1 << 20, 1, 1, rollout=64, sb=256)
    run(n199, 1 << 20, 1, 1, rollout=64, sb=1024)
