"""Precision probe: full MPPI updates of the oracle in fp64 Pinocchio-order
arithmetic vs fp64 world-frame zero-bias ABA vs fp32 dynamics, identical injected noise.

Usage: python tools/precision_probe.py SAMPLES HORISON [UPDATES]
"""
import os, sys, numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O
from assistedmanipulation_amd import config as cfg
m=O.default_model(); c=O.default_cost()
S,Hh=int(sys.argv[1]),float(sys.argv[2])
conf=cfg.frankaridgeback_configuration(rollouts=S, horison=Hh)
cc,keep=conf.to_c()
dyn=cfg.frankaridgeback_dynamics(m); cost=cfg.assisted_manipulation_cost(c)
trajs=[O.OracleTrajectory(cc,dyn,cost,scalar=s,mode=md) for (s,md) in [(0,0),(0,1),(1,1)]]
H=trajs[0].H
rng=np.random.default_rng(12345)
sd=np.sqrt(cfg.FR_VARIANCE)
x=cfg.huddled_state()
for t in trajs: t.set_forecast(cfg.constant_forecast(H))
for j in range(int(sys.argv[3]) if len(sys.argv)>3 else 5):
    time_=0.05*j
    n=trajs[0].noise_draws(time_)
    eps=rng.standard_normal((n,12))*sd
    for t in trajs:
        t.inject_noise(eps); t.update(x,time_)
    cs=[t.costs() for t in trajs]
    ref=cs[0]
    rng_=np.nanmax(ref)-np.nanmin(ref)
    print(f"upd {j}: cost range {np.nanmin(ref):.6e}..{np.nanmax(ref):.6e} nan={np.isnan(ref).sum()} argmin={[int(np.nanargmin(c_)) for c_ in cs]}")
    for name,c_ in zip(['red64','red32'],cs[1:]):
        d=np.abs(c_-ref)
        print(f"   {name}: max|d|={np.nanmax(d):.3e} max|d|/range={np.nanmax(d)/rng_:.3e} maxrel={np.nanmax(d/np.abs(ref)):.3e}")
    U=[t.optimal_control() for t in trajs]
    print("   U* diff red64 %.3e red32 %.3e (|U| %.3e)"%(np.abs(U[1]-U[0]).max(), np.abs(U[2]-U[0]).max(), np.abs(U[0]).max()))
    w=[t.weights() for t in trajs]
    print("   w diff red32 %.3e"%np.abs(w[2]-w[0]).max())
