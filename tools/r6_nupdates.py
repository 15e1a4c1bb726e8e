#!/usr/bin/env python3
"""Updates per env per env step of bench.py's config-5 workload (131,072 envs, Philox, the bench's
actions and attractors, per-step launches) from the CPU oracle -- input of tools/r6_sched_sim.py.
Trajectories are bit-exact with the GPU's, so these are the loop lengths the kernel runs.
Usage: python tools/r6_nupdates.py SPEC CAP T -> /tmp/sim/nup_SPEC_CAP.npy (SPEC: fixture | spec).
Measurement tooling only (imports the oracle)."""
import os
os.makedirs('/tmp/sim', exist_ok=True)
import sys, numpy as np, torch
R=os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0,R); sys.path.insert(0,R+'/oracle'); sys.path.insert(0,R+'/gym-pbn-stac_amd')
import oracle as O, bench
from gym_pbn_amd.network import load_network
from gym_pbn_amd.batch import EnvConfig, Net
from gym_pbn_amd.actions import env_actions
O.build()
spec, cap, T = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
B=131072
net=load_network('bittner199'); o=O.Oracle(net)
atts,_=bench.r6_attractors(spec, net.n_nodes)
cfg=EnvConfig(Net(net), atts, horizon=100)
cfgd=dict(care=cfg.cube_care, value=cfg.cube_value, target_care=cfg.target_care, target_value=cfg.target_value, horizon=100)
st,ns=o.env_reset_philox(np.zeros((B,net.n_words),np.uint64), np.ones(B,np.int64), cfg.reset_care, cfg.reset_value, seed=0xAC7, env_base=0, reset_count=0)
acts=env_actions(T,0,B,4,net.n_nodes,seed=0xAC7).numpy()
out=[]
for t in range(T):
    r=o.env_step_multi(cfgd, st, ns, acts[t], seed=0xAC7, env_base=0, call_idx=t, update_cap=cap)
    out.append(r['n_updates'].astype(np.uint32)); st,ns=r['state'],r['n_steps']
    print(t, out[-1].mean(), out[-1].max(), flush=True)
np.save(f'/tmp/sim/nup_{spec}_{cap}.npy', np.stack(out))
