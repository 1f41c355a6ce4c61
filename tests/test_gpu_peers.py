"""Upstream peer selection on the GPU through libgpumatch.so
(gm_peers_init / gm_select_peers / gm_release_peers) against the oracle's request-by-request
balancers (oracle/gm_oracle.c orc_select_peers), bit for bit: every pick and the whole balancer
state (conns, current_weight, flags) after every batch.

- the peers workload: every method, down peers, fallbacks, deferred upstreams, three batches
  with peers going down / coming back and connections released between them;
- 1M requests concentrated on a 70-peer round robin and a 67-peer least_conn upstream: the
  sequential kernels' periodic fill (k_peer_seq / k_peer_fill), with loaded peers
  (least_conn's catch-up phase before its period)."""

import numpy as np
import pytest

from gpumatch import engine, peers, records
from oracle_py import Balancer, Oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    assert torch.cuda.is_available(), "GPU test without a GPU"
    return torch, torch.device("cuda", 0)


class Gpu:
    def __init__(self, torch, dev, b, gen=1):
        self.torch, self.dev = torch, dev
        self.e = engine.Engine(0)
        self.e.load(b, gen)
        self.n_peers = self.e.stats()["n_peers"]
        self.state = torch.zeros(max(self.n_peers, 1) * 16, dtype=torch.uint8, device=dev)
        self.s = torch.cuda.current_stream().cuda_stream
        self.e.peers_init_ptr(self.state.data_ptr(), self.n_peers, self.s)

    def match_select(self, reqs, arena):
        t = self.torch
        n = len(reqs)
        d_reqs = t.from_numpy(np.ascontiguousarray(reqs).view(np.uint8).reshape(-1)).to(self.dev)
        d_arena = t.zeros(len(arena) + 1024, dtype=t.uint8, device=self.dev)
        d_arena[:len(arena)].copy_(t.from_numpy(np.ascontiguousarray(arena)))
        d_out = t.empty(n * 32, dtype=t.uint8, device=self.dev)
        cap = 4 * n + 1024
        d_hits = t.empty(cap, dtype=t.int32, device=self.dev)
        d_peer = t.full((n,), -7, dtype=t.int32, device=self.dev)
        self.e.match_ptr(d_reqs.data_ptr(), d_arena.data_ptr(), len(arena), n, d_out.data_ptr(), d_hits.data_ptr(),
                         cap, self.s)
        self.e.select_peers_ptr(d_reqs.data_ptr(), d_arena.data_ptr(), len(arena), n, d_out.data_ptr(),
                                self.state.data_ptr(), self.n_peers, d_peer.data_ptr(), self.s)
        self.e.sync(self.s)
        v = d_out.cpu().numpy().view(records.VERDICT_DTYPE)
        return v, d_peer.cpu().numpy().view(np.uint32)

    def state_np(self):
        self.torch.cuda.synchronize()
        return self.state.cpu().numpy().view(engine.PEER_STATE_DTYPE)[:self.n_peers].copy()

    def set_state(self, st):
        self.state[:self.n_peers * 16].copy_(self.torch.from_numpy(st.view(np.uint8).reshape(-1)))

    def release(self, ids):
        d = self.torch.from_numpy(np.ascontiguousarray(ids, dtype=np.uint32).view(np.int32)).to(self.dev)
        self.e.release_peers_ptr(d.data_ptr(), len(ids), self.state.data_ptr(), self.n_peers, self.s)


def _check(label, got, exp, gs, os_):
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, f"{label}: {len(bad)} picks differ; first i={bad[0]}: got {got[bad[0]]} exp {exp[bad[0]]}"
    for f in ("conns", "current_weight", "flags"):
        bad = np.nonzero(gs[f] != os_[f])[0]
        assert len(bad) == 0, f"{label}: state {f} differs at peers {bad[:8]}: {gs[f][bad[:8]]} vs {os_[f][bad[:8]]}"


def test_peer_selection_parity_batches(torch_dev):
    torch, dev = torch_dev
    b = peers.peers_blob()
    g = Gpu(torch, dev, b)
    o = Oracle(b, 1)
    bal = Balancer(o)
    assert g.n_peers == bal.n_peers
    _check("init", np.zeros(0), np.zeros(0), g.state_np(), bal.state)
    rng = np.random.default_rng(5)
    seen = set()
    for k in range(3):
        reqs, arena = peers.gen_requests(40_000, seed=records.SEED_BASE + 50 + k)
        v, got = g.match_select(reqs, arena)
        exp = bal.select(reqs, arena, v)
        _check(f"batch {k}", got, exp, g.state_np(), bal.state)
        seen.update(np.unique(got).tolist())
        # between batches: some peers go down / come back, some connections end
        st = g.state_np()
        flip = rng.choice(g.n_peers, 12, replace=False)
        st["flags"][flip] ^= engine.GM_PEER_DOWN
        bal.state["flags"][flip] ^= engine.GM_PEER_DOWN
        g.set_state(st)
        real = got[got < g.n_peers]
        rel = rng.choice(real, len(real) // 2, replace=False)
        g.release(rel)
        bal.release(rel)
        _check(f"after batch {k}", np.zeros(0), np.zeros(0), g.state_np(), bal.state)
    assert engine.GM_PEER_DEFER in seen and engine.GM_NONE in seen and len(seen) > 200


def test_peer_selection_long_sequential_runs(torch_dev):
    torch, dev = torch_dev
    b = peers.peers_blob()
    g = Gpu(torch, dev, b)
    o = Oracle(b, 1)
    bal = Balancer(o)
    # least_conn starts unbalanced: a catch-up phase before the state repeats
    st = g.state_np()
    st["conns"][:] = np.random.default_rng(9).integers(0, 40, g.n_peers)
    g.set_state(st)
    bal.state[:] = st
    for k in range(2):
        reqs, arena = peers.gen_requests(1_000_000, seed=records.SEED_BASE + 60 + k, hot=(1, 4))
        v, got = g.match_select(reqs, arena)
        exp = bal.select(reqs, arena, v)
        _check(f"1M batch {k}", got, exp, g.state_np(), bal.state)


def _expected_migration(e_old_addrs, old_state, e_new_addrs):
    """new peer j keeps the state of the first unused old peer of the same (address, upstream)."""
    used = set()
    out = np.zeros(len(e_new_addrs), dtype=engine.PEER_STATE_DTYPE)
    for j, key in enumerate(e_new_addrs):
        for i, k2 in enumerate(e_old_addrs):
            if k2 == key and i not in used:
                used.add(i)
                out[j] = old_state[i]
                break
    return out


def test_plus_endpoint_update_and_migration(torch_dev):
    """NGINX Plus endpoint updates (UpdateServersInPlus, configurator.go:442,467,489, no Reload):
    gm_update_upstream swaps one upstream's servers, gm_peers_migrate carries the balancer state
    (kept servers keep conns / current_weight / flags), and gm_select_peers then matches the
    oracle on the config a reload with the new server lines would have rendered, state included."""
    torch, dev = torch_dev
    b = peers.peers_blob()
    g = Gpu(torch, dev, b)
    o = Oracle(b, 1)
    bal = Balancer(o)
    reqs, arena = peers.gen_requests(40_000, seed=records.SEED_BASE + 70, hot=(1, 4, 9))
    v, got = g.match_select(reqs, arena)
    exp = bal.select(reqs, arena, v)
    _check("before the update", got, exp, g.state_np(), bal.state)
    servers = {}
    updates = [(1, [peers._addr(1, j) for j in range(5, 55)] + [f"10.77.0.{j}:9000" for j in range(1, 21)]),
               (9, [peers._addr(9, j) for j in (6, 0, 2)] + ["10.9.9.9:80"]),
               (4, [peers._addr(4, j) for j in range(0, 67, 2)] + ["10.4.9.1:8080"])]
    for k, (u, sv) in enumerate(updates):
        old_addrs = [g.e.peer_address(p) for p in range(g.n_peers)]
        old_state = g.state_np()
        old_n = g.n_peers
        g.e.update_upstream(peers.upstream_name(u), sv)
        servers[u] = peers.plus_order(servers.get(u, peers.server_addrs(u)), sv)
        st = g.e.stats()
        assert st["gen"] == 1   # configVersion unchanged by a Plus API update
        new_n = st["n_peers"]
        new_addrs = [g.e.peer_address(p) for p in range(new_n)]
        new_state = torch.zeros(max(new_n, 1) * 16, dtype=torch.uint8, device=dev)
        g.e.peers_migrate_ptr(g.state.data_ptr(), old_n, new_state.data_ptr(), new_n, g.s)
        g.state, g.n_peers = new_state, new_n
        exp_state = _expected_migration(old_addrs, old_state, new_addrs)
        _check(f"migration {k}", np.zeros(0), np.zeros(0), g.state_np(), exp_state)
        # the oracle on the re-rendered config, from the migrated state
        o2 = Oracle(peers.peers_blob(servers=servers), 1)
        bal2 = Balancer(o2)
        assert bal2.n_peers == new_n
        bal2.state[:] = exp_state
        reqs, arena = peers.gen_requests(40_000, seed=records.SEED_BASE + 71 + k, hot=(1, 4, 9))
        v, got = g.match_select(reqs, arena)
        exp = bal2.select(reqs, arena, v)
        _check(f"after update {k}", got, exp, g.state_np(), bal2.state)


BIG = [("hash $arg_user", 1500), ("hash $arg_user consistent", 1200), ("ip_hash", 1100), ("random", 1300),
       ("least_conn", 1500), ("", 3)]


def test_large_upstreams_round_robin_fallback(torch_dev):
    """a stateless method's round-robin fallback (empty hash key, > 20 down tries) in an
    upstream past k_peer_seq's LDS capacity (SEQ_PEERS_MAX = 1024 peers) defers to nginx instead
    of indexing past the LDS arrays; every other pick still matches the oracle."""
    torch, dev = torch_dev
    b = peers.peers_blob(upstreams=BIG)
    g = Gpu(torch, dev, b)
    o = Oracle(b, 1)
    bal = Balancer(o)
    reqs, arena = peers.gen_requests(60_000, seed=records.SEED_BASE + 80, upstreams=BIG)
    v, got = g.match_select(reqs, arena)
    exp = bal.select(reqs, arena, v)
    _check("big upstreams", got, exp, g.state_np(), bal.state)
    # the empty-key requests of the 1500-peer hash upstream deferred, the keyed ones picked
    up = v["upstream_id"]
    names = sorted(peers.upstream_name(u) for u in range(len(BIG) + 1))
    hid = names.index(peers.upstream_name(0))
    sel = (up == hid) & (v["action"] == 0)
    assert (got[sel] == engine.GM_PEER_DEFER).any() and (got[sel] < g.n_peers).any()


def test_sticky_cookie_parity(torch_dev):
    """NGINX Plus `sticky cookie` on the GPU (nginx-plus.ingress.tmpl:9-11,
    annotations.go:387-399): round robin, least_conn and random two least_conn upstreams with a
    srv_<k> cookie naming a peer by the hex MD5 of its address -- present, naming a down peer,
    stale, malformed, another upstream's, absent -- every pick and the whole state equal the
    oracle's over two batches with peers going down between them.  Parity unpinned (no Plus)."""
    torch, dev = torch_dev
    b = peers.sticky_blob()
    g = Gpu(torch, dev, b)
    o = Oracle(b, 1)
    bal = Balancer(o)
    assert g.n_peers == bal.n_peers and g.e.stats()["n_upstreams_deferred"] == 0
    for k, down in enumerate([(), (1, 4, 9)]):
        st = bal.state.copy()
        st["flags"][:] = 0
        st["flags"][list(down)] = 1
        bal.state[:] = st
        g.set_state(st)
        reqs, arena = peers.sticky_requests(60_000, seed=records.SEED_BASE + 300 + k)
        v, got = g.match_select(reqs, arena)
        ev, _ = o.match(reqs, arena)
        assert np.array_equal(v, ev)
        exp = bal.select(reqs, arena, ev)
        _check(f"sticky batch {k}", got, exp, g.state_np(), bal.state)
    assert (got < g.n_peers).sum() > 40_000
