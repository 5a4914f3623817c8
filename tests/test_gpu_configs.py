"""BASELINE.json configs 2-4 at full size on ONE MI355X, through the in-process rank group.

The reference cannot run any of them (`int` N, mpi_radix_sort.c:65, mpi_sample_sort.c:33;
Zipf bucket overflow, mpi_sample_sort.c:144,167 -- SURVEY.md 8 Q12), so parity here is by
size-independent properties, checked on device (K9):
  * the multiset fingerprint (sum and xor of mix64(key)) of all outputs == of all inputs,
  * every rank's output is sorted and rank q's last key <= rank q+1's first key,
  * radix: rank q holds exactly global positions [qB, (q+1)B) (B = ceil(N/P));
  * sample: the per-rank sizes equal the bucket counts the ranks exchanged.
Inputs are the canonical splitmix64 stream generated on device, rank r holding
keys [rB, (r+1)B) of it -- the same stream the oracle and bench.py use.  Each case prints the
receive imbalance (largest rank / N/P).
"""
import threading

import pytest

pytestmark = pytest.mark.gpu

MASK64 = (1 << 64) - 1


def run_generated(gsort, P, n_total, dist, algo, seed=42, balanced=False):
    grp = gsort.Group(P)
    B = -(-n_total // P)
    res, errs = [None] * P, []

    def worker(r):
        try:
            with gsort.Context(rank=r, group=grp) as c:
                c.set_sample_balanced(balanced)
                n = max(0, min(B, n_total - r * B))
                p = c.alloc(max(n, 1) * 4)
                c.generate(dist, seed, r * B, n, p)
                fin = c.fingerprint(p, n)
                out, m, st = (c.radix if algo == "radix" else c.sample)(p, n)
                fout = c.fingerprint(out, m)
                info = c.sample_info() if algo == "sample" else None
                res[r] = {"n_in": n, "n_out": m, "fin": fin, "fout": fout, "stats": st,
                          "info": info}
                c.free(p)
        except Exception as e:  # surfaced in the main thread
            errs.append((r, e))

    th = [threading.Thread(target=worker, args=(r,), daemon=True) for r in range(P)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=900)
    hung = [r for r, t in enumerate(th) if t.is_alive()]
    if hung:
        pytest.fail(f"ranks {hung} did not finish")
    grp.close()
    if errs:
        print("\n".join(f"rank {r}: {e}" for r, e in errs))
        raise errs[0][1]
    return res, B


def check_global_order(res, n_total):
    s_in = x_in = s_out = x_out = 0
    for r in res:
        s_in = (s_in + r["fin"]["sum"]) & MASK64
        x_in ^= r["fin"]["xor"]
        s_out = (s_out + r["fout"]["sum"]) & MASK64
        x_out ^= r["fout"]["xor"]
        assert r["fout"]["sorted"]
    assert (s_out, x_out) == (s_in, x_in), "output multiset != input multiset"
    assert sum(r["n_out"] for r in res) == n_total
    nonempty = [r for r in res if r["n_out"]]
    for a, b in zip(nonempty, nonempty[1:]):
        assert a["fout"]["last"] <= b["fout"]["first"], "ranks out of order"


def imbalance(res, n_total):
    P = len(res)
    return max(r["n_out"] for r in res) / (n_total / P)


@pytest.mark.parametrize("P", [2, 4, 8])
def test_config2_radix_2p31(gsort, P):
    """configs[2]: radix sort of 2^31 uniform keys across 2/4/8 ranks (one exchange, exact
    splitters): rank q ends with global positions [qB, (q+1)B)."""
    n = 1 << 31
    res, B = run_generated(gsort, P, n, gsort.UNIFORM, "radix")
    check_global_order(res, n)
    assert [r["n_out"] for r in res] == [min(B, n - q * B) for q in range(P)]
    assert all(r["stats"]["exchanges"] == 1 for r in res)
    print(f"\nconfigs[2] P={P}: imbalance {imbalance(res, n):.4f}, "
          f"max pair {max(r['stats']['max_pair_bytes'] for r in res)} B")


@pytest.mark.parametrize("P", [2, 4, 8])
def test_config3_sample_2p30(gsort, P):
    """configs[3]: sample sort of 2^30 uniform keys at 2/4/8 ranks (regular sampling, device
    splitter selection, one exchange of exact sizes)."""
    n = 1 << 30
    res, B = run_generated(gsort, P, n, gsort.UNIFORM, "sample")
    check_global_order(res, n)
    # rank q's size = the column sum of the exchanged P x P bucket matrix
    for q in range(P):
        assert res[q]["n_out"] == sum(int(res[r]["info"][1][q]) for r in range(P))
    ib = imbalance(res, n)
    print(f"\nconfigs[3] P={P}: imbalance {ib:.4f}")
    # the reference's rule on uniform keys: rank r's 2P-1 samples sit at the quantiles
    # j/(2P-1) of its block, so the sorted P(2P-1) samples hold each quantile P times and
    # s[i] = S[(i+1)(2P-1)] (mpi_sample_sort.c:123) is the quantile floor((i+1)(2P-1)/P)/(2P-1);
    # rank q receives the keys between s[q-1] and s[q]
    k = 2 * P - 1
    cut = [0.0] + [((i + 1) * k // P) / k for i in range(P - 1)] + [1.0]
    for q in range(P):
        assert abs(res[q]["n_out"] / n - (cut[q + 1] - cut[q])) < 0.01, (q, res[q]["n_out"])


@pytest.mark.parametrize("balanced", [False, True])
def test_config4_sample_zipf_2p32_p8(gsort, balanced):
    """configs[4]: sample sort of 2^32 Zipf (s = 1.5) keys on 8 ranks.  The reference's bucket
    rule (balanced=False) puts every copy of the hot key on one rank (~30 % of all keys, where
    the reference overflows its fixed buckets); the duplicate-aware rule shares them out."""
    P, n = 8, 1 << 32
    res, B = run_generated(gsort, P, n, gsort.ZIPF, "sample", balanced=balanced)
    check_global_order(res, n)
    ib = imbalance(res, n)
    print(f"\nconfigs[4] balanced={balanced}: imbalance {ib:.3f} "
          f"(largest rank {max(r['n_out'] for r in res)} keys)")
    if balanced:
        assert ib < 1.6
    else:
        assert max(r["n_out"] for r in res) > 0.25 * n
