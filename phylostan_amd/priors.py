"""Tree priors and hyper-priors of the emitted Stan models, with gradients.

Restatements of the Stan functions ``phylostan/generate_script.py`` emits:

* ``constant_coalescent_log``  ``:285-349``
* ``skyride_coalescent_log``   ``:352-419``
* ``skygrid_coalescent_log``   ``:422-500``
* ``gmrf_log``                 ``:606-619``  (not time-aware)

Each takes node ``times`` (internal nodes: heights, tips: sampling ages),
an ``internal`` mask and the population parameters, for a batch of draws
(leading axis ``n``), and returns ``(logP [n], grads...)``.  The event order
is ``argsort(times)`` (Stan: ``sort_indices_asc``); zero-length intervals
contribute nothing, as in the Stan code's ``if (interval != 0.0)``.
"""
import math

import numpy as np


def _sorted_events(times, internal):
    order = np.argsort(times, axis=1, kind="stable")
    t = np.take_along_axis(times, order, axis=1)
    intl = internal[order]
    # lineages present during the interval that ends at event i
    step = np.where(intl, -1.0, 1.0)
    k = np.cumsum(step, axis=1) - step
    c = k * (k - 1.0) * 0.5
    dt = np.diff(t, axis=1, prepend=t[:, :1])
    return order, t, intl, c, dt


def _scatter_back(order, g_sorted):
    g = np.empty_like(g_sorted)
    np.put_along_axis(g, order, g_sorted, axis=1)
    return g


def constant_coalescent(times, internal, theta):
    """``heights ~ constant_coalescent(theta, map[, lowers])``.

    times [n, N], internal bool [N], theta [n] -> (logP [n], dtimes [n, N], dtheta [n])."""
    order, t, intl, c, dt = _sorted_events(times, internal)
    nz = dt != 0.0
    inv = 1.0 / theta
    a = np.where(nz, c, 0.0)
    lp = -(dt * a).sum(axis=1) * inv - intl.sum(axis=1) * np.log(theta)
    # d/dt_i: interval i ends at t_i (coef -a_i), interval i+1 starts there (+a_{i+1})
    nxt = np.concatenate([a[:, 1:], np.zeros((a.shape[0], 1))], axis=1)
    gs = (nxt - a) * inv[:, None]
    dtheta = (dt * a).sum(axis=1) * inv * inv - intl.sum(axis=1) * inv
    return lp, _scatter_back(order, gs), dtheta


def skyride_coalescent(times, internal, pop):
    """``heights ~ skyride_coalescent(thetas, map[, lowers])`` with log
    population sizes ``pop [n, S-1]`` (one per coalescent interval)."""
    order, t, intl, c, dt = _sorted_events(times, internal)
    nz = dt != 0.0
    adv = nz & intl
    idx = np.cumsum(adv, axis=1) - adv  # pop index in force at event i
    idx = np.minimum(idx, pop.shape[1] - 1)
    lpop = np.take_along_axis(pop, idx, axis=1)
    e = np.exp(-lpop)
    a = np.where(nz, c * e, 0.0)
    lp = -(dt * a).sum(axis=1) - np.where(adv, lpop, 0.0).sum(axis=1)
    nxt = np.concatenate([a[:, 1:], np.zeros((a.shape[0], 1))], axis=1)
    gs = nxt - a
    gpop = np.zeros_like(pop)
    rows = np.broadcast_to(np.arange(pop.shape[0])[:, None], idx.shape)
    np.add.at(gpop, (rows, idx), np.where(nz, dt * a, 0.0) - adv)
    return lp, _scatter_back(order, gs), gpop


def skygrid_coalescent(times, internal, pop, grid):
    """``heights ~ skygrid_coalescent(thetas, map, grid[, lowers])``:
    ``pop [n, G]`` log sizes on the grid ``grid [G]`` (event loop)."""
    n, N = times.shape
    G = len(grid)
    lp = np.zeros(n)
    gtimes = np.zeros_like(times)
    gpop = np.zeros_like(pop)
    for d in range(n):
        order = np.argsort(times[d], kind="stable")
        t = times[d][order]
        intl = internal[order]
        index = 0
        lps = pop[d, 0]
        ps = math.exp(lps)
        start = t[0]
        start_var = 0  # sorted position of the event `start` equals, or -1 for a grid point
        k = 0.0
        for i in range(N):
            finish = t[i]
            c = k * (k - 1.0) * 0.5
            while index < G - 1 and finish > grid[index]:
                end = min(grid[index], finish)
                end_var = i if grid[index] >= finish else -1
                w = c / ps
                lp[d] -= (end - start) * w
                gpop[d, index] += (end - start) * w
                if end_var >= 0:
                    gtimes[d, order[end_var]] -= w
                if start_var >= 0:
                    gtimes[d, order[start_var]] += w
                start, start_var = end, end_var
                index += 1
                lps = pop[d, index]
                ps = math.exp(lps)
            w = c / ps
            lp[d] -= (finish - start) * w
            gpop[d, index] += (finish - start) * w
            gtimes[d, order[i]] -= w
            if start_var >= 0:
                gtimes[d, order[start_var]] += w
            if intl[i]:
                lp[d] -= lps
                gpop[d, index] -= 1.0
                k -= 1.0
            else:
                k += 1.0
            start, start_var = finish, i
    return lp, gtimes, gpop


def gmrf(logpop, precision):
    """``thetas ~ gmrf(tau)`` (not time-aware): returns (logP, dlogpop, dprecision)."""
    N = logpop.shape[1]
    d = np.diff(logpop, axis=1)
    s = (d * d).sum(axis=1)
    lp = np.log(precision) * (N - 1.0) / 2.0 - s * precision / 2.0 - (N - 1.0) / 2.0 * math.log(2.0 * math.pi)
    gd = -precision[:, None] * d
    glog = np.zeros_like(logpop)
    glog[:, 1:] += gd
    glog[:, :-1] -= gd
    gprec = (N - 1.0) / (2.0 * precision) - s / 2.0
    return lp, glog, gprec
