"""Diagnostic: config-2 GPU vs oracle, every pass, with the exchange record."""
import sys, numpy as np, torch
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests")
import abnn_amd
from oracle import oracle as O
from shard_helpers import GpuShards

def mk_g():
    g = abnn_amd.Brain(256, 256, 99_488, 10_000_000, 10_000_000); g.build_random_graph(1)
    g.set_auto_stimulus(0, 256); return g
o = O.OracleBrain(256, 256, 99_488, 10_000_000, 10_000_000); o.build_random_graph(1, nthreads=16)
o.set_auto_stimulus(0, 256)
g = mk_g(); h = mk_g(); sh = GpuShards([h])
words = o.exchange_words(); rec = np.zeros(words, dtype=np.int32)
for k in range(8):
    if k == 7:
        for b in (g, h, o): b.set_reward(-0.25)
    o2 = None
    g.encode_traversal(1); sh.pass_(); torch.cuda.synchronize()
    o.pass_threaded(nthreads=16)
    gr = sh.gathered.cpu().numpy()
    syn_g, syn_h = g.download_synapses().view(np.uint32), h.download_synapses().view(np.uint32)
    so = o.syn.view(np.uint32)
    lf_g, lf_h, lf_o = g.last_fired(), h.last_fired(), o.last_fired
    print(k, "syn g/o", int((syn_g.reshape(-1) != so.reshape(-1)).sum()),
          "syn h/o", int((syn_h.reshape(-1) != so.reshape(-1)).sum()), "lf g/o", int((lf_g != lf_o).sum()), "lf h/o", int((lf_h != lf_o).sum()),
          "summary", gr[:8].view(np.int64).tolist(), "g", g.stats(), "o", o.stats(), flush=True)
    if (lf_g != lf_o).any():
        idx = np.nonzero(lf_g != lf_o)[0][:10]
        print("  lf idx", idx.tolist(), lf_g[idx].tolist(), lf_o[idx].tolist())
        n = int(gr[:2].view(np.int64)[0]); sp = gr[8:8 + n]
        print("  spikes n", n, "unique", len(np.unique(sp)), "max", int(sp.max()) if n else -1, "min", int(sp.min()) if n else -1)
