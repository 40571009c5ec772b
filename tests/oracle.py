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
