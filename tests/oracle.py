"""Independent fp64 NumPy replay of the reference engines (math only, given arrival sets)."""
import numpy as np

from erasurehead_amd.models.losses import LOGISTIC, UpdateRule, worker_grad


def replay(scheme, parts, beta0, arrivals_log, rule, alpha, n_samples, eta, kind=LOGISTIC):
    """parts: list of (X, y) numpy.  Returns betaset [R, d] following ref src/*.py updates."""
    up = UpdateRule("AGD" if scheme.fixed_agd else rule, alpha, n_samples, scheme.grad_scale())
    beta = np.array(beta0, dtype=np.float64)
    u = np.zeros_like(beta)
    out = []
    from erasurehead_amd.codes.schemes import Arrival

    for i, arr in enumerate(arrivals_log):
        arrivals = [Arrival(w, p, t) for (w, p, t) in arr]
        used = scheme.decode(arrivals)
        g = np.zeros_like(beta)
        for (w, part), c in used.items():
            m = [x for x in scheme.messages if x.worker == w and x.part == part][0]
            msg = sum(worker_grad(kind, parts[p][0], parts[p][1], beta, coef) for p, coef in m.segments)
            g += c * msg
        up.apply(i, eta[i], beta, u, g)
        out.append(beta.copy())
    return np.array(out)


def stops_exactly_at_last(scheme, arrivals_log):
    """The stop rule (csrc/runtime/collector.h kinds) holds after the last logged arrival of every
    round and after no earlier one: a collector that kept books wrongly would log late arrivals or
    stop early.  arrivals_log: [[(worker, part, ...), ...] per round]."""
    from erasurehead_amd.codes.schemes import RULE_ALL, RULE_COUNT, RULE_FRC, RULE_PARTIAL_COUNT, RULE_PARTIAL_FRC

    kind, k = scheme.rule()
    W, G = scheme.n_workers, scheme.n_groups

    def holds(c0, c1, cg):
        return {RULE_ALL: c0 >= W, RULE_COUNT: c0 >= k, RULE_FRC: c0 >= k or cg >= G,
                RULE_PARTIAL_FRC: c1 >= W and cg >= G, RULE_PARTIAL_COUNT: c1 >= W and c0 >= k}[kind]

    for arr in arrivals_log:
        got0, got1, groups = set(), set(), set()
        states = []
        for a in arr:
            w, p = int(a[0]), int(a[1])
            if p == 0:
                got0.add(w)
                groups.add(scheme.group_of[w])
            else:
                got1.add(w)
            states.append(holds(len(got0), len(got1), len(groups)))
        if not states or not states[-1] or any(states[:-1]):
            return False
    return True
