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
    if x0 is not None:  # osqp_warm_start: x / D, y / E * c, z = A x (scaled)
        x=np.asarray(x0,float)/D; y=np.asarray(y0,float)/E*c if y0 is not None else y; z=A@x
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


class OSQP:
    """The same dense restatement with osqp-python's object API for a receding-horizon loop
    (OSQP 0.6 semantics the reference's scripts rely on): scaling (D, E, c) computed once at
    setup from (P, q, A) and kept; update(q=, l=, u=) scales the new vectors with it and
    re-classifies the rho vector (refactor when a row changes class); x, z, y (scaled) and the
    adapted rho persist from one solve to the next, and a warm-started solve starts from them.
    solve() returns x, y (unscaled) and info.status / info.iter.  Test infrastructure only."""

    def setup(self, P, q, A, l, u, rho=0.1, sigma=1e-6, alpha=1.6, eps_abs=1e-3, eps_rel=1e-3, max_iter=4000,
              scaling=10, check_termination=25, adaptive_rho_interval=0, adaptive_rho_tolerance=5,
              warm_start=True, verbose=False, **_):
        P = np.triu(P.toarray() if hasattr(P, "toarray") else np.asarray(P)).astype(float)
        A = (A.toarray() if hasattr(A, "toarray") else np.asarray(A)).astype(float)
        q = np.asarray(q, float).copy()
        n, m = P.shape[0], A.shape[0]
        D = np.ones(n); E = np.ones(m); c = 1.0
        Pf = lambda Pu: Pu + np.triu(Pu, 1).T  # noqa: E731
        for _ in range(scaling):
            Pful = Pf(P)
            Dt = np.maximum(np.abs(Pful).max(0), np.abs(A).max(0) if m else 0)
            Et = np.abs(A).max(1)
            Dt = 1 / np.sqrt(limit(Dt)); Et = 1 / np.sqrt(limit(Et))
            P = Dt[:, None] * P * Dt[None, :]; A = Et[:, None] * A * Dt[None, :]; q = Dt * q
            D *= Dt; E *= Et
            ct = np.abs(Pf(P)).max(0).mean()
            nq = limit(np.array([np.abs(q).max()]))[0]
            ct = max(ct, nq); ct = limit(np.array([ct]))[0]; ct = 1 / ct
            P *= ct; q *= ct; c *= ct
        self.Pful, self.A, self.q, self.D, self.E, self.c = Pf(P), A, q, D, E, c
        self.n, self.m = n, m
        self.sigma, self.alpha, self.eps_abs, self.eps_rel, self.max_iter = sigma, alpha, eps_abs, eps_rel, max_iter
        self.check = check_termination
        self.interval = adaptive_rho_interval or (4 * check_termination if check_termination else 100)
        self.tol, self.warm = adaptive_rho_tolerance, warm_start
        self.rho = min(max(rho, RHO_MIN), RHO_MAX)
        self._bounds(l, u)
        self.x = np.zeros(n); self.z = np.zeros(m); self.y = np.zeros(m)

    def _bounds(self, l, u):
        l = np.maximum(np.asarray(l, float), -INF); u = np.minimum(np.asarray(u, float), INF)
        self.l, self.u = self.E * l, self.E * u
        self.rv = self._rhovec(self.rho)
        self.Kinv = self._factor(self.rv)

    def _rhovec(self, rho):
        r = np.where(self.u - self.l < RHO_TOL, EQ * rho, rho)
        return np.where((self.l < -INF * MINS) & (self.u > INF * MINS), RHO_MIN, r)

    def _factor(self, rv):
        return np.linalg.inv(self.Pful + self.sigma * np.eye(self.n) + self.A.T @ (rv[:, None] * self.A))

    def update(self, q=None, l=None, u=None):
        if q is not None:
            self.q = self.c * (self.D * np.asarray(q, float))
        if l is not None or u is not None:
            lo = self.l / self.E if l is None else l
            up = self.u / self.E if u is None else u
            self._bounds(lo, up)

    def solve(self):
        from types import SimpleNamespace
        A, Pful, q, D, E, c = self.A, self.Pful, self.q, self.D, self.E, self.c
        sigma, alpha = self.sigma, self.alpha
        if not self.warm:
            self.x = np.zeros(self.n); self.z = np.zeros(self.m); self.y = np.zeros(self.m)
        x, z, y, rv, Kinv = self.x, self.z, self.y, self.rv, self.Kinv
        status = "maximum iterations reached"
        # (check iteration, max(prim_res / eps_prim, dual_res / eps_dual)) of every termination
        # check: the solve stops at the first ratio below 1 -- how close each decision was
        self.last_checks = []
        for k in range(1, self.max_iter + 1):
            xp, zp = x, z
            xt = Kinv @ (sigma * xp - q + A.T @ (rv * zp - y)); zt = A @ xt
            x = alpha * xt + (1 - alpha) * xp
            z = np.clip(alpha * zt + (1 - alpha) * zp + y / rv, self.l, self.u)
            y = y + rv * (alpha * zt + (1 - alpha) * zp - z)
            chk = self.check and k % self.check == 0
            ad = k % self.interval == 0
            if chk or ad:
                Ax = A @ x; Px = Pful @ x; Aty = A.T @ y
                if chk:
                    pr = np.abs((Ax - z) / E).max(); dr = np.abs((Px + q + Aty) / D).max() / c
                    ep = self.eps_abs + self.eps_rel * max(np.abs(z / E).max(), np.abs(Ax / E).max())
                    ed = self.eps_abs + self.eps_rel * max(np.abs(q / D).max(), np.abs(Aty / D).max(),
                                                           np.abs(Px / D).max()) / c
                    self.last_checks.append((k, max(pr / ep, dr / ed)))
                    if pr < ep and dr < ed:
                        status = "solved"
                        break
                if ad:
                    prs = np.abs(Ax - z).max() / (max(np.abs(z).max(), np.abs(Ax).max()) + 1e-30)
                    drs = np.abs(Px + q + Aty).max() / (max(np.abs(q).max(), np.abs(Aty).max(), np.abs(Px).max()) + 1e-30)
                    rn = self.rho * np.sqrt(prs / (drs + 1e-30)); rn = min(max(rn, RHO_MIN), RHO_MAX)
                    if rn > self.rho * self.tol or rn < self.rho / self.tol:
                        self.rho = rn; rv = self._rhovec(rn); Kinv = self._factor(rv)
        self.x, self.z, self.y, self.rv, self.Kinv = x, z, y, rv, Kinv
        return SimpleNamespace(x=D * x, y=E * y / c, info=SimpleNamespace(status=status, iter=k))
