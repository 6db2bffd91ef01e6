"""CPU check of the as-intended window fold's float screens (maveric-slam_amd/csrc/hip/k_frontend.hip,
window_fold): outside its margins the float decision must equal the exact integer one, for the
threshold (the initial best (81 |q|^2, 100)) and for "beats the best" (d^2 n_b > d_b^2 n), over
random and adversarial (near-tie) operands in the kernel's ranges: |dot|, |a|^2, |q|^2 <= 256 * 128^2.
The GPU computes each product in float32 with round-to-nearest, as numpy does here."""
import numpy as np

F = np.float32
MAXN = 256 * 128 * 128  # 256 int8 products


def screen(d, n, bq, bn):
    """the kernel's float screen: returns (win, ambiguous) for candidate (d, n) against best (bq, bn)"""
    fd2 = F(d) * F(d)
    L = F(fd2 * F(bn))
    R = F(F(bq) * F(n))
    win = L > F(R * F(1.000002))
    amb = (not win) and L >= F(R * F(0.999998))
    return bool(win), bool(amb)


def exact_beats(d, n, bd2, bn):
    return d * d * bn > bd2 * n


def test_screen_never_contradicts_the_exact_order():
    rng = np.random.default_rng(11)
    bad = 0
    checked = 0
    for _ in range(200000):
        n = int(rng.integers(1, MAXN))
        q2 = int(rng.integers(1, MAXN))
        d = int(rng.integers(1, int(np.sqrt(n * q2)) + 1))  # Cauchy-Schwarz: d^2 <= n q2
        # against the threshold (the initial best): (d_b^2, n_b) = (81 q2, 100)
        win, amb = screen(d, n, F(81.0) * F(q2), 100)
        if not amb:
            checked += 1
            bad += win != exact_beats(d, n, 81 * q2, 100)
        # against a real best (db, nb) near the candidate's score
        nb = int(rng.integers(1, MAXN))
        db = int(round(d * np.sqrt(nb / n) * (1 + rng.normal(0, 1e-6))))
        db = max(1, db)
        win, amb = screen(d, n, F(db) * F(db), nb)
        if not amb:
            checked += 1
            bad += win != exact_beats(d, n, db * db, nb)
    assert bad == 0 and checked > 250000, (bad, checked)


def test_exact_ties_are_always_ambiguous():
    """equal scores (m w against m' w, and threshold-equal cosines) must reach the exact path"""
    rng = np.random.default_rng(12)
    for _ in range(20000):
        w = rng.integers(-20, 21, 8)
        q = rng.integers(-20, 21, 8)
        if (w @ q) <= 0:
            continue
        m1, m2 = (int(x) for x in rng.integers(1, 7, 2))
        d1, n1 = int(m1 * (w @ q)), int(m1 * m1 * (w @ w))
        d2, n2 = int(m2 * (w @ q)), int(m2 * m2 * (w @ w))
        win, amb = screen(d2, n2, F(d1) * F(d1), n1)
        assert amb and not win  # a tie is never a float "win"
    # threshold-equal: u = (0, 1, 1), v = (-3, 4, 5) scaled -- 100 d^2 == 81 |v|^2 |u|^2
    for ku in range(1, 9):
        for kv in range(1, 5):
            d, n, q2 = 9 * ku * kv, 50 * kv * kv, 2 * ku * ku
            assert 100 * d * d == 81 * n * q2
            win, amb = screen(d, n, F(81.0) * F(q2), 100)
            assert amb and not win
