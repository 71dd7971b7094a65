"""Edge cases of the lean kernels' compact cells (NPAD = 64, sender peers; brc_internal.h C32_*):
send steps stored as 7-bit offsets from a per-item epoch that moves past step 100, no slot
generations (a slot's 64-cell row is rewritten fresh at every allocation: PROPOSE, a consensus
SEND, an injected SEND / KEY), and set sizes that saturate at 63.  Every case is checked bit-exact against the C oracle (or against the engine's own
first pass for repeated resets, whose first pass the oracle pins)."""
import pytest

from oracle import oracle
from tests import golden_io
from tests.golden import specs as S

pytestmark = pytest.mark.gpu

ALL64 = (1 << 64) - 1


@pytest.fixture(scope="module")
def runner():
    from tests import engine_runner
    return engine_runner


def _check(got, specs):
    for sp, r in zip(specs, got):
        exp = oracle.run(sp)
        exp["events"] = golden_io.canonical_events(exp["events"])
        for k in ("status", "t_stop", "msgs_sent", "arrivals", "cell_steps"):
            assert r[k] == exp[k], "%s %s: %r vs oracle %r" % (sp["name"], k, r[k], exp[k])
        for k in ("deliver", "decide", "send"):
            assert r["events"][k] == exp["events"][k], "%s: %s events differ" % (sp["name"], k)


@pytest.mark.parametrize("model,dmax,rcap", [(1, 5, 8), (3, 6, 14)])
def test_spec_coin_rounds_reallocate_rows_and_move_epochs(runner, model, dmax, rcap):
    """SPEC (common coin) at n = 64 with Q = 2: each round reallocates both slots of an origin
    (every allocation rewrites the slot's row, so no stale cell of the previous round may
    survive it) and the runs pass step 190 (the epoch moves twice)."""
    specs = []
    for g in range(2):
        sp = S.spec_cons_spec(64, 21, 0x5EC64, model, dmax, 700 + g, round_cap=rcap, window=2, coin_seed=0xC0C0)
        sp["name"] = "lean-spec/%d" % g
        specs.append(sp)
    got = runner.run_specs(specs)
    _check(got, specs)
    assert max(r["t_stop"] for r in got) > 190


def test_epoch_moves_under_open_cells(runner):
    """Cells that stay open (no quorum) keep send steps from before two epoch moves; later
    messages of the same key must not match those old steps (an aliased 7-bit step would add
    arrivals).  Byzantine replicas 58..63 drive one key over 900 steps."""
    n, f = 64, 21
    byz = list(range(58, 64))
    kp = 60
    few = sum(1 << d for d in range(0, 10))            # the SEND reaches replicas 0..9 only
    acts = [dict(t=0, kind="byz_key", kp=kp, s=0, value=1),
            dict(t=0, kind="byz", src=60, type=S.SEND, kp=kp, s=0, dst=few),
            dict(t=3, kind="byz", src=61, type=S.ECHO, kp=kp, s=0, dst=ALL64),
            dict(t=120, kind="byz", src=62, type=S.ECHO, kp=kp, s=0, dst=ALL64),
            dict(t=121, kind="byz", src=58, type=S.READY, kp=kp, s=0, dst=ALL64),
            dict(t=245, kind="byz", src=63, type=S.ECHO, kp=kp, s=0, dst=ALL64),
            dict(t=247, kind="byz", src=59, type=S.READY, kp=kp, s=0, dst=ALL64),
            dict(t=900, kind="byz", src=60, type=S.ECHO, kp=kp, s=0, dst=ALL64),
            dict(t=901, kind="byz", src=61, type=S.READY, kp=kp, s=0, dst=ALL64)]
    specs = []
    for g in range(2):
        sends = [(0, 0, 0), (118, 1, 0), (126, 2, 0), (246, 3, 0), (899, 4, 0)]
        sp = S.brb_spec(n, f, 0xE90C, 2 if g == 0 else 1, 8 if g == 0 else 6, 90 + g, sends, byzantine=byz,
                        extra=acts)
        sp["name"] = "lean-epoch/%d" % g
        specs.append(sp)
    got = runner.run_specs(specs)
    _check(got, specs)
    assert all(r["t_stop"] > 900 for r in got)


def test_repeated_resets_rewrite_rows():
    """Ten reset + run passes over one engine (cfg4 shape, 8 instances): brc_reset leaves the
    previous pass's cells in place and every slot is reallocated (its row rewritten fresh) in
    each pass; each pass must equal the first, which the oracle pins."""
    from byzantinerandomizedconsensus_amd import _lib as L
    from byzantinerandomizedconsensus_amd.engine import Engine
    specs = [S.cons_spec(64, 21, 0x5EED0004, 2, 8, 5000 + g, round_cap=1) for g in range(8)]
    for i, sp in enumerate(specs):
        sp["name"] = "lean-reset/%d" % i
    first = None
    with Engine(n=64, f=21, instances=8, seed=0x5EED0004, delay_model=L.DELAY_SLOWSET, delay_max=8,
                round_cap=1, key_window=4, proposals=L.PROPOSALS_PHILOX, instance_offset=5000,
                event_capacity=1 << 20) as eng:
        for p in range(10):
            if p:
                eng.reset()
            eng.run()
            res = eng.instances_result()
            reps = eng.replicas()
            evs = sorted(map(tuple, eng.events()))
            snap = (res, reps, evs)
            if first is None:
                first = snap
                for sp, r in zip(specs, res):
                    exp = oracle.run(sp)
                    for k in ("status", "t_stop", "msgs_sent", "arrivals", "cell_steps"):
                        assert r[k] == exp[k], "%s %s" % (sp["name"], k)
            else:
                assert snap == first, "pass %d differs from the first" % p


# Q = 4 holds one round of phase indices (a second round reuses slots still in flight: BRC_OVERFLOW,
# which the oracle does not model), Q = 8 two rounds
@pytest.mark.parametrize("nv,window,rcap", [(1, 4, 1), (1, 8, 2), (2, 4, 1)])
def test_reference_consensus_windows_and_variants_vs_oracle(runner, nv, window, rcap):
    """Reference-protocol consensus on the lean kernel with each key window and, with two key
    variants, equivocating Byzantine senders: the consensus pass takes a word's deliveries at
    once when they can change no phase (fold_groups / compress_groups over Q * NV slots per
    origin) and one by one otherwise; both must equal the oracle's message-by-message run."""
    n, f = 40, 13
    byz = list(range(35, 40)) if nv == 2 else []
    specs = []
    for g in range(12):
        sp = S.cons_spec(n, f, 0xB01C + window, 0 if g % 2 else 2, 1 if g % 2 else 8, 4100 + g, round_cap=rcap,
                         byzantine=byz, nv=nv, extra=S.equivocation_actions(n, byz) if byz else ())
        sp["name"] = "lean-cons-q%d-nv%d/%d" % (window, nv, g)
        specs.append(sp)
    groups = {}
    for sp in specs:                                     # one batch per delay model (consecutive ids)
        groups.setdefault(sp["delay_model"], []).append(sp)
    for batch in groups.values():
        got = []
        for sp in batch:                                 # ids are not consecutive inside a model group
            got += runner.run_batch([sp], key_window=window)
        _check(got, batch)


@pytest.mark.parametrize("window,model,dmax", [(4, 1, 3), (8, 2, 8), (8, 3, 6)])
def test_spec_consensus_word_at_once_vs_oracle(runner, window, model, dmax):
    """SPEC consensus on the lean kernel (n = 48): the consensus pass adds a word's deliveries to
    the phase-slot counts at once when every delivering lane is at one phase index and none can
    complete its phase, one by one otherwise; coin rounds keep phases apart across replicas."""
    specs = []
    for g in range(8):
        sp = S.spec_cons_spec(48, 15, 0x5EC48 + window, model, dmax, 900 + g, round_cap=3, window=window,
                              coin_seed=0xC0DE)
        sp["name"] = "lean-spec-bulk-q%d/%d" % (window, g)
        specs.append(sp)
    got = runner.run_specs(specs)
    _check(got, specs)
