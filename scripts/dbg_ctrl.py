import sys, numpy as np
sys.path[:0]=['/root/repo','/root/repo/gym-flock_amd']
from gym_flock import _native as nat
from oracle import flocking as orc
n=40
rs=np.random.RandomState(9)
base=rs.uniform(-2,2,size=(n,4))
cases=[]
x=base.copy(); x[1,:2]=x[0,:2]; cases.append(("coincident",x))
x=base.copy(); x[:,1]=0.0; x[:,0]=np.arange(n)*0.9; cases.append(("boundary",x))
x=base.copy(); x[:,:2]+=3.0e5; cases.append(("huge",x))
x=base.copy(); x[5,0]=np.inf; cases.append(("inf",x))
for name,x0 in cases:
    u=rs.uniform(-1,1,size=(n,2)).astype(np.float32)
    out=[]
    for fl in (0, nat.FE_WITH_CONTROLLER):
        h=nat.FlockHandle(n,1); h.set_state(x0[None]); h.step(u[None], fl)
        out.append(h.state_values(0)); h.close()
    with np.errstate(all="ignore"):
        ref=orc.step(x0,u,with_controller=True)["state_values"]
    for lab,sv in (("plain",out[0]),("ctrl",out[1])):
        ok=~np.isnan(ref)
        bad=np.where(np.any(~np.isclose(sv,ref,rtol=1e-5,atol=1e-9)&ok,axis=1))[0]
        print(name, lab, "bad rows", bad[:20], len(bad))
