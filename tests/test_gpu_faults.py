"""Infrastructure failures must never read as rejections. SmartBFT treats any
VerifyProposal error as a Byzantine leader (complain, sync, abort: internal/bft/view.go:386-393)
and a failed vote as a bad signature (view.go:839-841), so the plugin has to tell "the engine
could not verify" (a negative SBFT_GV_E* code, -1 .. -6; the Go binding turns it into fail-stop)
apart from "the signature is invalid" (SBFT_V_EVERIFY, -10).

The engine's test-only fault injection (sbft_gv_inject_fault) fails its allocation, launch and
synchronisation points on demand. Every entry point on the hot path -- VerifyProposal (generic
and registered-client launches), VerifyConsenterSigs, the processCommits mirror, the coalesced
and the single VerifyConsenterSig, VerifyRequest, the prev-commit hook -- must then return an
engine code, never EVERIFY and never a wrong verdict, and the context must work again on the
next call once the fault is disarmed."""
import threading

import pytest

from smartbft_amd import plugin
from smartbft_amd.gpuverify import FAULT_LAUNCH, FAULT_NOMEM, FAULT_OFF, FAULT_SYNC, inject_fault

from test_gpu_plugin import _priv, _proposal

pytestmark = pytest.mark.gpu

KINDS = {"nomem": FAULT_NOMEM, "launch": FAULT_LAUNCH, "sync": FAULT_SYNC}


def _engine_code(code: int) -> bool:
    return -6 <= code <= -1


@pytest.fixture(scope="module")
def fnet():
    from smartbft_amd import GpuVerifier
    gv = GpuVerifier(device_mask=1)
    nodes = [plugin.Signer(gv, i, _priv(("fault", i))) for i in range(1, 8)]
    v = plugin.Verifier(gv, verification_sequence=3)
    for s in nodes:
        v.add_consenter(s.id, s.public_key())
    clients = [plugin.Signer(gv, 2000 + i, _priv(("fclient", i))) for i in range(8)]
    vr = plugin.Verifier(gv, verification_sequence=3)  # all clients registered: the keyed launch
    vr.add_clients([c.public_key() for c in clients])
    yield gv, v, vr, nodes, clients
    inject_fault(FAULT_OFF)
    for o in [v, vr] + nodes + clients:
        o.close()
    gv.close()


def _calls(v, vr, nodes, clients):
    """Each hot-path entry point as (name, thunk returning a comparable result)."""
    p, reqs = _proposal(clients, 1200)
    sigs = [n.SignProposal(p, b"aux%d" % n.id) for n in nodes]
    dig = p.Digest()

    def coalesced():
        v.coalesce_consenter_sigs(16, 2000)
        out, errs = [None] * len(sigs), []

        def one(i):
            try:
                out[i] = v.VerifyConsenterSig(sigs[i], p)
            except plugin.VerifyError as e:
                errs.append(e)
        th = [threading.Thread(target=one, args=(i,)) for i in range(len(sigs))]
        for t in th:
            t.start()
        for t in th:
            t.join()
        v.coalesce_consenter_sigs(1, 0)
        if errs:
            raise errs[0]
        return out

    return [
        ("VerifyProposal", lambda: [(i.ClientID, i.ID) for i in v.VerifyProposal(p)]),
        ("VerifyProposal-registered", lambda: [(i.ClientID, i.ID) for i in vr.VerifyProposal(p)]),
        ("VerifyConsenterSigs", lambda: v.VerifyConsenterSigs(sigs, p)),
        ("collect_commits", lambda: v.collect_commits([(s, dig) for s in sigs], p, need=5)[0]),
        ("VerifyConsenterSig", lambda: v.VerifyConsenterSig(sigs[0], p)),
        ("VerifyConsenterSig-coalesced", coalesced),
        ("VerifyRequest", lambda: (lambda i: (i.ClientID, i.ID))(v.VerifyRequest(reqs[5]))),
        ("prev_commit_signatures", lambda: v.verify_prev_commit_signatures(sigs, p, curr_vseq=3)),
    ]


@pytest.mark.parametrize("kind", list(KINDS))
def test_engine_faults_are_not_verdicts(fnet, kind):
    gv, v, vr, nodes, clients = fnet
    calls = _calls(v, vr, nodes, clients)
    want = {name: f() for name, f in calls}  # healthy engine, warmed up
    failed = []
    for name, f in calls:
        inject_fault(KINDS[kind], -1)  # every fault point of this kind fails
        try:
            got = f()
        except plugin.VerifyError as e:
            assert _engine_code(e.code), f"{name}: {kind} fault surfaced as verdict code {e.code}: {e}"
            assert e.code != plugin.EVERIFY
            failed.append(name)
        else:  # a path without a fault point of this kind must still be right
            assert got == want[name], f"{name}: wrong result under a {kind} fault"
        finally:
            inject_fault(FAULT_OFF)
        assert f() == want[name], f"{name}: the context did not recover after a {kind} fault"
    # every path has at least one fault point of every kind it can meet: launches everywhere
    if kind == "launch":
        assert sorted(failed) == sorted(n for n, _ in calls), failed
    else:
        assert failed, f"no entry point reached a {kind} fault point"


def test_one_shot_fault_then_recovery(fnet):
    """count = 1: exactly one fault point fails; the call reports it and the very next call
    through the same context succeeds with the same verdicts."""
    gv, v, vr, nodes, clients = fnet
    p, _ = _proposal(clients, 300, tamper=123)
    with pytest.raises(plugin.VerifyError) as ei:
        v.VerifyProposal(p)
    assert ei.value.code == plugin.EVERIFY and ei.value.index == 123
    inject_fault(FAULT_LAUNCH, 1)
    try:
        with pytest.raises(plugin.VerifyError) as ei:
            v.VerifyProposal(p)
        assert _engine_code(ei.value.code) and ei.value.index is None
    finally:
        inject_fault(FAULT_OFF)
    with pytest.raises(plugin.VerifyError) as ei:
        v.VerifyProposal(p)
    assert ei.value.code == plugin.EVERIFY and ei.value.index == 123


def test_init_rejects_reserved_fields():
    """sbft_gv_opts' reserved fields must be 0: a caller still setting a retired field (reserved0
    was quad_max) gets SBFT_GV_EINVAL instead of having it read as something else."""
    import ctypes
    from smartbft_amd.gpuverify import Opts, load_library
    L = load_library()
    for field in ("reserved0", "reserved1"):
        o = Opts()
        o.device_mask = 1
        setattr(o, field, 1)
        ctx = ctypes.c_void_p()
        assert L.sbft_gv_init(ctypes.byref(o), ctypes.byref(ctx)) == -1, field
        assert not ctx.value
