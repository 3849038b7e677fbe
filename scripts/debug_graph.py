"""Debug: config-5 batches, eager vs eager (determinism) and graph replay vs eager, per output."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from orleans_amd import workloads as W
from orleans_amd.engine import GrainDirectoryEngine

n_games, per_game, n_hb = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000, 8, 64 * 1024
cl = W.default_cluster()
pr = W.presence_population(n_games, per_game)
n_keys = n_games * (1 + per_game)
all_keys = np.concatenate([pr.game_keys, pr.player_keys])
owner = cl.owner_of(W.jenkins3_np(all_keys["tcd"], all_keys["n0"], all_keys["n1"]))
n_fan = n_hb * per_game
eng = GrainDirectoryEngine(n_act=n_keys, dir_capacity=n_keys, max_batch=n_fan, device=0)
W.setup_engine(eng, cl)
W.register_population(eng, all_keys, owner, np.ones(n_keys, bool))
batches = [W.heartbeat_batch(pr, cl, n_hb, b) for b in range(3)]
dev = "cuda"
d_msgs = [torch.from_numpy(m.view(np.int32).reshape(-1, 8)).to(dev) for _, m in batches]
d_games = [torch.from_numpy(g.view(np.int32)).to(dev) for g, _ in batches]
d_gsilo = [torch.from_numpy(owner[g.astype(np.int64)]).to(dev) for g, _ in batches]
d_off = torch.from_numpy(pr.csr_off.view(np.int64)).to(dev)
d_tgt = torch.from_numpy(pr.csr_tgt.view(np.int32)).to(dev)
d_pkeys = torch.from_numpy(pr.player_keys.view(np.uint8).reshape(-1, 24)).to(dev)
o1 = [torch.empty(n_hb, dtype=torch.int32, device=dev) for _ in range(3)]
o2 = [torch.empty(n_fan, dtype=torch.int32, device=dev) for _ in range(3)]
off1 = torch.empty(n_keys + 2, dtype=torch.int32, device=dev)
off2 = torch.empty(n_keys + 2, dtype=torch.int32, device=dev)
poff = torch.empty(n_hb + 1, dtype=torch.int64, device=dev)
s = torch.cuda.Stream()
sp = s.cuda_stream
outs = o1 + o2 + [off1, off2]
names = ["route1", "act1", "order1", "route2", "act2", "order2", "off1", "off2"]


def one(i, mode):
    if mode in ("both", "route"):
        eng.address_messages_device(d_msgs[i], n_hb, o1[0], o1[1], o1[2], off1, stream=sp)
    if mode in ("both", "fan"):
        eng.fanout_keys_device(d_off, d_tgt, d_pkeys, d_games[i], d_gsilo[i], n_hb, poff, o2[0], o2[1], o2[2], off2,
                               stream=sp, total=n_fan)


def snap():
    s.synchronize()
    return [x.clone() for x in outs]


def diff(a, b, tag):
    bad = [(nm, int((x != y).sum())) for nm, x, y in zip(names, a, b) if not torch.equal(x, y)]
    print(tag, "OK" if not bad else bad, flush=True)


for mode in ("route", "fan", "both"):
    with torch.cuda.stream(s):
        one(0, mode); one(1, mode)
    e1 = None
    with torch.cuda.stream(s):
        one(1, mode)
    e1 = snap()
    with torch.cuda.stream(s):
        one(0, mode); one(1, mode)
    diff(e1, snap(), f"[{mode}] eager(1) vs eager(0),eager(1)")
    graphs = []
    for i in range(2):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            one(i, mode)
        graphs.append(g)
    s.synchronize()
    for i in range(2):
        for x in outs:
            x.fill_(-1)
        torch.cuda.synchronize()
        with torch.cuda.stream(s):
            graphs[i].replay()
        rep = snap()
        with torch.cuda.stream(s):
            one(i, mode)
        diff(rep, snap(), f"[{mode}] graph({i}) vs eager({i})")
    del graphs
eng.close()
