"""ReferenceSchedule (train_step.py) against train.py:388-414 on a recording stand-in trainer (CPU:
the schedule is host logic; the trainer's densify / prune kernels are covered by the GPU tests)."""
import pytest

from train_step import ReferenceSchedule


class _Rec:
    def __init__(self, P):
        self.P, self.calls = P, []

    def densify(self, g, o, extent, size):
        self.calls.append(("densify", g, o, extent, size))
        self.P += 1000

    def prune(self, g, o, extent, size):
        self.calls.append(("prune", g, o, extent, size))
        self.P -= 10

    def reset_opacity(self):
        self.calls.append(("reset",))


def test_neu3d_defaults_fire_on_the_reference_iterations():
    tr, s = _Rec(100_000), ReferenceSchedule(extent=2.0)
    for it in range(1, 1001):
        s(tr, it)
    # densify after 500 every 100 while P < 360000; prune only once P > 200000
    assert [c[0] for c in tr.calls] == ["densify"] * 5
    assert [e[0] for e in s.events] == [600, 700, 800, 900, 1000]
    assert all(c[1:] == ("densify", 2e-4, 0.005, 2.0, None)[1:] for c in tr.calls)


def test_prune_size_threshold_and_reset():
    tr = _Rec(250_000)
    s = ReferenceSchedule(extent=1.0, opacity_reset_interval=700, densify_until_iter=1000,
                          opacity_threshold_fine_init=0.01, opacity_threshold_fine_after=0.0)
    for it in range(1, 1000):
        s(tr, it)
    names = [e[:2] for e in s.events]
    assert [e[0] for e in s.events if e[1] == "reset_opacity"] == [700]
    prunes = [c for c in tr.calls if c[0] == "prune"]
    assert prunes[0][4] is None and prunes[-1][4] == 20          # size threshold once past the reset interval
    # the opacity threshold interpolates init -> after over densify_until_iter
    assert prunes[0][2] == pytest.approx(0.01 - 600 / 1000 * 0.01)


def test_no_statistics_or_events_after_densify_until_iter():
    tr, s = _Rec(100_000), ReferenceSchedule(extent=1.0, densify_until_iter=700)
    assert s.collect_stats(699) and not s.collect_stats(700)
    for it in range(1, 2000):
        s(tr, it)
    assert [e[0] for e in s.events] == [600]
    assert not ReferenceSchedule(extent=1.0, stage="fine-lang").collect_stats(10)
