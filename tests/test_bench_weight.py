"""bench.py's choice of rank 0's share of the row split (choose_root_weight): 1 while
the ranks' gathers keep up with their renders, a larger share for rank 0 — whose rows never
cross a link — when the peers' gathers are link-bound."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import choose_root_weight  # noqa: E402


def test_fast_links_keep_the_equal_split():
    assert choose_root_weight(8, [0.0048] * 8, [0.002] * 8) == 1
    assert choose_root_weight(4, [0.0096] * 4, [0.0099] * 4) == 1   # within the margin
    assert choose_root_weight(1, [0.038], [0.0]) == 1


def test_link_bound_peers_shift_rows_to_rank0():
    # 2 ranks, each peer frame share 3.1 MB at ~60 GB/s: 51 us of gather against 19 us of render
    w = choose_root_weight(2, [0.0193, 0.0193], [0.051, 0.051])
    assert w == 3
    T, L = 0.0386, 0.102
    V = w + 1
    assert max(T * w / V, max(T, L) / V) < 0.6 * max(T / 2, L / 2)
    assert choose_root_weight(8, [0.0048] * 8, [0.0128] * 8) >= 2


def test_link_estimate_is_the_fastest_peer():
    # rank 0's gather waits for the slowest peer and one peer waited for rank 0: the fastest
    # peer's gather is the link time
    assert choose_root_weight(4, [0.0096] * 4, [0.05, 0.0101, 0.03, 0.0099]) == 1
    assert choose_root_weight(2, [0.0193] * 2, [0.2, 0.051]) == 3


def test_degenerate_probes():
    assert choose_root_weight(4, [], []) == 1
    assert choose_root_weight(4, [0.0, 0.01, 0.01, 0.01], [0.05] * 4) == 1
