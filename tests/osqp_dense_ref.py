"""Independent dense numpy restatement of the OSQP 0.6 iteration -- TEST INFRASTRUCTURE.

A second, deliberately different implementation (dense matrices, explicit
inverse of the reduced KKT matrix P + sigma I + A' diag(rho) A) used to pin the
C oracle (oracle/osqp_oracle.c): both must produce the same iterates, so status,
iteration count and x agree to rounding.  Cold start, scaling on, pinned
adaptive-rho interval (see oracle/osqp_oracle.h).
"""
import numpy as np
INF=1e30; MINS=1e-4; MAXS=1e4; RHO_MIN=1e-6; RHO_MAX=1e6; RHO_TOL=1e-4; EQ=1e3
def limit(v):
    v=np.where(v<MINS,1.0,v); return np.where(v>MAXS,MAXS,v)
def solve(P,q,A,l,u,rho=0.1,sigma=1e-6,alpha=1.6,eps_abs=1e-3,eps_rel=1e-3,max_iter=4000,scaling=10,check=25,interval=100,tol=5,x0=None,y0=None,verbose=False):
    P=np.triu(P).astype(float); A=A.astype(float); q=q.astype(float).copy()
    l=np.maximum(l,-INF); u=np.minimum(u,INF)
    n=P.shape[0]; m=A.shape[0]
    D=np.ones(n); E=np.ones(m); c=1.0
    Pf=lambda Pu: Pu+np.triu(Pu,1).T
    for it in range(scaling):
        Pful=Pf(P)
        Dt=np.maximum(np.abs(Pful).max(0), np.abs(A).max(0) if m else 0)
        Et=np.abs(A).max(1)
        Dt=1/np.sqrt(limit(Dt)); Et=1/np.sqrt(limit(Et))
        P=Dt[:,None]*P*Dt[None,:]; A=Et[:,None]*A*Dt[None,:]; q=Dt*q
        D*=Dt; E*=Et
        ct=np.abs(Pf(P)).max(0).mean()
        nq=limit(np.array([np.abs(q).max()]))[0]
        ct=max(ct,nq); ct=limit(np.array([ct]))[0]; ct=1/ct
        P*=ct; q*=ct; c*=ct
    l=E*l; u=E*u
    Pful=Pf(P)
    rho=min(max(rho,RHO_MIN),RHO_MAX)
    def rhovec(rho):
        r=np.where(u-l<RHO_TOL, EQ*rho, rho)
        r=np.where((l<-INF*MINS)&(u>INF*MINS), RHO_MIN, r)
        return r
    rv=rhovec(rho)
    def factor(rv): return np.linalg.inv(Pful+sigma*np.eye(n)+A.T@(rv[:,None]*A))
    Kinv=factor(rv)
    x=np.zeros(n); z=np.zeros(m); y=np.zeros(m)
    status='max_iter'; nref=0
    for k in range(1,max_iter+1):
        xp=x; zp=z
        xt=Kinv@(sigma*xp-q+A.T@(rv*zp-y)); zt=A@xt
        x=alpha*xt+(1-alpha)*xp
        z=np.clip(alpha*zt+(1-alpha)*zp+y/rv,l,u)
        dy=rv*(alpha*zt+(1-alpha)*zp-z); y=y+dy
        chk=(k%check==0); ad=(k%interval==0)
        if chk or ad:
            Ax=A@x; Px=Pful@x; Aty=A.T@y
            pr=np.abs((Ax-z)/E).max(); dr=np.abs((Px+q+Aty)/D).max()/c
            if chk:
                ep=eps_abs+eps_rel*max(np.abs(z/E).max(),np.abs(Ax/E).max())
                ed=eps_abs+eps_rel*max(np.abs(q/D).max(),np.abs(Aty/D).max(),np.abs(Px/D).max())/c
                if pr<ep and dr<ed: status='solved'; break
            if ad:
                prs=np.abs(Ax-z).max()/(max(np.abs(z).max(),np.abs(Ax).max())+1e-30)
                drs=np.abs(Px+q+Aty).max()/(max(np.abs(q).max(),np.abs(Aty).max(),np.abs(Px).max())+1e-30)
                rn=rho*np.sqrt(prs/(drs+1e-30)); rn=min(max(rn,RHO_MIN),RHO_MAX)
                if rn>rho*tol or rn<rho/tol:
                    rho=rn; rv=rhovec(rho); Kinv=factor(rv); nref+=1
    return D*x, E*y/c, status, k, nref
