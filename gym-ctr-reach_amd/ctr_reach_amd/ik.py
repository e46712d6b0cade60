"""Batched damped-least-squares position IK on the GPU Jacobian.

Restates ``dls_ik_position_only`` (ctr_reach_envs/src/jacobian_controller.py:19-73) for a batch
of targets: every iteration takes the forward-difference Jacobian J and the tip P of the env's
forward kinematics (CtrReachVecEnv.jacobian, one ctr_jacobian launch for the whole batch), then

    e  = P_d - P
    q += J^T (J J^T + lam I)^-1 e
    stop (per target) once |e| < tol          (checked after the update, as the reference does)

The reference builds a CTR_Model (its BVP model) for J; here J is the env's own FK
(model.py:30-70), so the IK is consistent with the environment the policy acts in.  Plotting
is omitted.  A target whose iterate leaves the nesting constraints into a tube gap (NaN FK; the
reference's solver loops forever there) stops at its last finite iterate with err = NaN.
"""


def dls_ik_position_only(env, targets, q0, system=None, lam=0.25, num=500, tol=1e-3, eps=1e-4):
    """targets [M, 3], q0 [M, 6] (float64 tensors or arrays) -> (q [M, 6], err [M], iters [M])."""
    import torch
    dev = env.device
    pd = torch.as_tensor(targets, dtype=torch.float64, device=dev).reshape(-1, 3)
    q = torch.as_tensor(q0, dtype=torch.float64, device=dev).reshape(-1, 6).clone()
    m = q.shape[0]
    sys_t = None if system is None else torch.as_tensor(system, dtype=torch.int32, device=dev).reshape(-1).expand(m)
    active = torch.ones(m, dtype=torch.bool, device=dev)
    err = torch.full((m,), float("inf"), dtype=torch.float64, device=dev)
    iters = torch.zeros(m, dtype=torch.int32, device=dev)
    eye = lam * torch.eye(3, dtype=torch.float64, device=dev)
    for _ in range(int(num)):
        idx = torch.nonzero(active).flatten()
        if idx.numel() == 0:
            break
        s = None if sys_t is None else sys_t[idx]
        p, jac = env.jacobian(q[idx], s, eps=eps)
        e = pd[idx] - p
        bad = ~torch.isfinite(e).all(dim=1) | ~torch.isfinite(jac).flatten(1).all(dim=1)
        if bool(bad.any()):
            # the iterate left the nesting constraints into a tube gap (NaN FK, where the
            # reference's solver never returns): stop that target at its last finite iterate
            err[idx[bad]] = float("nan")
            active[idx[bad]] = False
            keep = ~bad
            idx, p, jac, e = idx[keep], p[keep], jac[keep], e[keep]
            if idx.numel() == 0:
                continue
        jjt = jac @ jac.transpose(1, 2) + eye
        dq = (jac.transpose(1, 2) @ torch.linalg.solve(jjt, e.unsqueeze(-1))).squeeze(-1)
        q[idx] += dq
        en = torch.linalg.norm(e, dim=1)
        err[idx] = en
        iters[idx] += 1
        active[idx] = en >= tol
    return q, err, iters
