"""Host-only: the axis-aligned quad test's accept bounds (rt_flatten.cpp accept_interval,
rt_layout.h). The device accepts a hit when the hit point's in-plane coordinates y lie in
[y0, y1] (or are NaN); the reference accepts when a = (y - q) * C lies in [0, 1] (or is NaN),
object.rs:469-473 in the reduced form a = pq_i A_i. Each bound pair the generated walker carries
must be exactly the edge of that set: both bounds accepted by the reference's arithmetic, their
outside neighbours rejected. q, C are restated here in Python f64 (IEEE, no fusion) from the
blob's own q, u, v, w, as the flattener forms them."""
import math
import re

import numpy as np

import surely_rt as rt

RT_OBJ_LIST, RT_OBJ_QUAD = 1, 4


def _f64(slot):
    return float(np.uint64(slot).view(np.float64))


def _quads(blob):
    """(q, u, v, w) of the world list's quads, in order (include/rt_mi355x.h blob layout)."""
    s = blob.slots
    p = blob.header()["world_off"]
    assert int(s[p]) == RT_OBJ_LIST
    n = int(s[p + 1])
    p += 2 + 6
    out = []
    for _ in range(n):
        assert int(s[p]) == RT_OBJ_QUAD
        f = [_f64(s[p + 2 + k]) for k in range(17)]
        out.append((f[0:3], f[3:6], f[6:9], f[12:15]))
        p += 2 + 17 + 6
    return out


def _accept(y, q, c):
    a = (y - q) * c
    return not (a < 0.0) and not (1.0 < a)


def test_generated_bounds_are_the_exact_edges_of_the_reference_accept_set():
    sc = rt.Scene(5)
    m = sc.lambertian((0.5, 0.5, 0.5))
    specs = [  # odd sizes, negative edges, off-grid origins, all three normal axes
        ((0.1, -3.7, 2.25), (0, 1.3, 0), (0, 0, -7.1)),
        ((555, 0, 0), (0, 555, 0), (0, 0, 555)),
        ((213, 554, 227), (130, 0, 0), (0, 0, 105)),
        ((-1e-3, 7.77, 1e3), (0, 0, 3.3e-2), (-0.61, 0, 0)),
        ((12.5, 1e-7, -4.0), (0.3, 0, 0), (0, 2.0 / 3.0, 0)),
        ((0, 0, 0), (1e-9, 0, 0), (0, 5e3, 0)),
    ]
    world = sc.hittable_list(*[sc.quad(q, u, v, m) for q, u, v in specs])
    blob = sc.serialize(world, None)
    state, src = rt.jit_check(blob)
    assert state == 1
    lits = re.findall(r"aquad_test<COUNT, (\d)>\(AQuad\{\d+u, ([^,]+), ([^,]+), ([^,]+), ([^,]+), "
                      r"([^}]+)\}", src)
    quads = _quads(blob)
    assert len(lits) == len(quads) == len(specs)
    for (k_s, *vals), (q, u, v, w) in zip(lits, quads):
        qk, lo0, lo1, hi0, hi1 = (float.fromhex(x.strip("() ")) for x in vals)
        i = next(c for c in range(3) if u[c] != 0.0)
        j = next(c for c in range(3) if v[c] != 0.0)
        k = 3 - i - j
        assert int(k_s) == k and qk == q[k]
        # A = v x w, B = w x u (rt_flatten.cpp), one component each
        A = (v[1] * w[2] - v[2] * w[1], v[2] * w[0] - v[0] * w[2], v[0] * w[1] - v[1] * w[0])
        B = (w[1] * u[2] - w[2] * u[1], w[2] * u[0] - w[0] * u[2], w[0] * u[1] - w[1] * u[0])
        axes = sorted([(i, q[i], A[i]), (j, q[j], B[j])])
        for (_, qa, ca), (y0, y1) in zip(axes, [(lo0, lo1), (hi0, hi1)]):
            assert y0 <= y1
            assert _accept(y0, qa, ca) and _accept(y1, qa, ca)
            assert not _accept(math.nextafter(y0, -math.inf), qa, ca)
            assert not _accept(math.nextafter(y1, math.inf), qa, ca)
            # interior points and the NaN convention
            for t in np.linspace(0.0, 1.0, 17):
                assert _accept(y0 + (y1 - y0) * float(t), qa, ca) or t in (0.0, 1.0)
            assert _accept(math.nan, qa, ca)
