#!/usr/bin/env python3
"""Wave-scheduling model of one R6 per-step launch of k_env (mode 4) at config 5's size, driven by
the real loop lengths (tools/r6_nupdates.py). Per workgroup of 4 waves x 64 lanes (one env per lane at
131,072 envs): lane mode runs 32-update chunks for every live env (c_chunk + draw rounds), a wave with
the queue dry and <= tail_max live envs resolves them one at a time in 64-update tail blocks (c_blk,
c_sess per env step, longest-used first), handing envs it has not started to idle sibling waves
(c_push) at session start and every 16 blocks. Returns the predicted kernel ms (max over workgroups).
Calibrated on the measured per-step lines (c_chunk = 32 x 0.25 us, c_blk = 0.7 us: 1.30 / 2.15 /
0.53 ms predicted vs 1.26-1.29 / 2.12-2.21 / 0.49-0.51 measured for the 4,096 cap / cap 2^20 / the
spec attractors); `python tools/r6_sched_sim.py /tmp/sim/nup_*.npy` prints the base prediction and the
policy sweep quoted in DESIGN.md §6 (round 4). Measurement tooling only."""
import numpy as np, sys, math
def simulate(nup, P, tail_max=16, long_first=True, lanes=64, wg_waves=4, handoff=True, order='lowest'):
    """nup: updates per env for one env step (B envs). Returns predicted kernel ms."""
    B=len(nup); nw=B//lanes
    ends=[]
    for g in range(nw//wg_waves):
        waves=[]
        for w in range(wg_waves):
            base=(g*wg_waves+w)*lanes
            envs=[[int(nup[base+k]),0] for k in range(lanes)]  # [remaining, used]
            waves.append({'envs':envs,'t':P['t0'],'tail':False,'idle':False,'drained':False})
        # event loop: always advance the non-idle wave with the smallest t
        while True:
            act=[w for w in waves if not w['idle']]
            if not act: break
            W=min(act,key=lambda w:w['t'])
            E=[e for e in W['envs'] if e[0]>0]
            W['envs']=E
            if not E:
                W['idle']=True; W['t_idle']=W['t']; continue
            if not W['tail'] and W['drained'] and len(E)<=tail_max: W['tail']=True
            if not W['tail']:
                n=len(E)
                dt=P['c_chunk'] + P['c_draw']*(math.ceil(n*16/64) if n<40 else 8)
                for e in E:
                    p=min(32,e[0]); e[0]-=p; e[1]+=p
                W['t']+=dt
                if any(e[0]==0 for e in E) or True: W['drained']=True
                continue
            # tail session: choose env
            if long_first and any(e[1]>=1024 for e in E):
                i=max(range(len(E)),key=lambda k:(E[k][1],-k))
            else: i=0
            env=E[i]; others=[e for k,e in enumerate(E) if k!=i]
            def push():
                nonlocal others
                if not handoff: return
                idle=[w for w in waves if w['idle'] and w is not W]
                for w in idle:
                    if not others: break
                    e=others.pop()  # the highest lanes go
                    w['envs']=[e]; w['idle']=False; w['tail']=True; w['drained']=True
                    w['t']=max(w['t_idle'],W['t'])+P['c_push']
            push()
            W['envs']=[env]+others
            W['t']+=P['c_sess']
            nb=math.ceil(env[0]/64)
            # 16-block segments; a segment's end may find new idle siblings
            while nb>0:
                s=min(16,nb); W['t']+=s*P['c_blk']; nb-=s
                if nb>0:
                    W['envs']=[env]+others
                    # other waves may have gone idle before W['t']: let them catch up first
                    for w in waves:
                        if w is W or w['idle']: continue
                    push()
            env[1]+=env[0]; env[0]=0
            W['envs']=others
        ends.append(max(w['t'] for w in waves))
    return max(ends)/1e3, np.percentile(ends,50)/1e3
if __name__=='__main__':
    base=dict(t0=20.0,c_chunk=32*0.25,c_draw=0.25,c_blk=0.7,c_sess=2.0,c_push=1.0)
    D={f:np.load(f) for f in sys.argv[1:]}
    def run(label, **kw):
        P=dict(base); P.update(kw.pop('P',{}))
        print(f'{label:28s}', {f.split('/')[-1]: round(float(np.mean([simulate(n[t],P,**kw)[0] for t in range(min(3,n.shape[0]))])),3)
                               for f,n in D.items()}, flush=True)
    run('base (tail 16)')
    run('no hand-off', handoff=False)
    for tm in (24,32): run(f'tail {tm}', tail_max=tm)
    for cb in (0.5,0.35):
        for tm in (16,32): run(f'c_blk {cb} tail {tm}', tail_max=tm, P=dict(c_blk=cb))
    run('lane 0.2 us/update', P=dict(c_chunk=32*0.2))
    run('8-wave hand-off pool', wg_waves=8)
