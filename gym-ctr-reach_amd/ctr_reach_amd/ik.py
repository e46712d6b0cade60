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


def dls_ik_position_only(env, targets, q0, system=None, lam=0.25, num=500, tol=1e-3, eps=1e-4, check_every=8):
    """targets [M, 3], q0 [M, 6] (float64 tensors or arrays) -> (q [M, 6], err [M], iters [M]).

    The iteration is stream-ordered: every iteration runs on the whole batch with finished targets
    masked out, and the host reads the "any target still active" flag only every
    ``check_every`` iterations (to stop early), so the loop does not synchronise per iteration."""
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
    nan = torch.tensor(float("nan"), dtype=torch.float64, device=dev)
    for k in range(int(num)):
        if k % max(1, int(check_every)) == 0 and not bool(active.any()):
            break
        p, jac = env.jacobian(q, sys_t, eps=eps)
        e = pd - p
        # an iterate that left the nesting constraints into a tube gap (NaN FK, where the
        # reference's solver never returns) stops at its last finite iterate with err = NaN
        bad = active & (~torch.isfinite(e).all(dim=1) | ~torch.isfinite(jac).flatten(1).all(dim=1))
        err = torch.where(bad, nan, err)
        live = active & ~bad
        jl = torch.where(live[:, None, None], jac, torch.zeros_like(jac))
        el = torch.where(live[:, None], e, torch.zeros_like(e))
        jjt = jl @ jl.transpose(1, 2) + eye
        dq = (jl.transpose(1, 2) @ torch.linalg.solve(jjt, el.unsqueeze(-1))).squeeze(-1)
        q = torch.where(live[:, None], q + dq, q)
        en = torch.linalg.norm(el, dim=1)
        err = torch.where(live, en, err)
        iters = iters + live.to(torch.int32)
        active = live & (en >= tol)
    return q, err, iters
