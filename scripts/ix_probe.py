import sys, numpy as np
sys.path.insert(0, "/root/repo")
from sitewhere_amd.persistence import segments as sg
from sitewhere_amd.pipeline.bus_io import RawBatchRecord, parse_raw_batch
from sitewhere_amd.pipeline.config import EngineConfig
from sitewhere_amd.pipeline.fleet import FleetSpec, fingerprints, gen_payloads, gen_tokens, stamp_alt_epoch
from sitewhere_amd.pipeline.framing import varint_lengths
from sitewhere_amd.pipeline.gpu_engine import GpuInboundEngine
n_dev = 1 << 20
heap, offs = gen_tokens("dev-", 0, n_dev)
lo, hi = fingerprints(heap, offs)
spec = FleetSpec(prefix="dev-", n_devices=n_dev, p_location=0.25, p_alert=0.05, p_unregistered=0.005, with_alternate_id=True)
now = 1_700_000_001_000
base = [gen_payloads(spec, 1 << 20, now - 30_000, seed=11 + b) for b in range(2)]
def nalt(blk):
    toff = sg.trailer_offset(blk)
    return int(sg.parse_trailer(blk[toff:])["n_alt"]), int(blk[:64].view(sg.HDR)[0]["n_rows"])
for filt in (0, 1 << 24):
    for framed in (False, True):
        cfg = EngineConfig(max_msgs=1 << 20, rec_cap=(1 << 20) + 4096, gen_cap=1 << 19, max_devices=n_dev + 65536,
                           max_assignments=n_dev + 65536, store_cap=1 << 23, dedup_slots=1 << 22, name_slots=1 << 12,
                           state_slots=1 << 24, dedup_filter_ids=filt, dedup_filter_gens=4)
        g = GpuInboundEngine(cfg, device="cuda:0")
        d = g.register_devices(lo, hi); g.set_assignments(d, d)
        g.encode_blocks, g.block_boot = True, 0x5eed
        res = []
        for k in range(4):
            raw, off = base[k % 2]
            raw = np.concatenate([raw, np.zeros(64, np.uint8)])
            stamp_alt_epoch(raw, off, (0x50AC << 48) | k)
            if framed:
                rec = RawBatchRecord(raw[:int(off[-1])], varint_lengths(off), len(off) - 1, pinned=True)
                res += [(k, r.block.copy(), rec) for _, r in g.submit_framed(parse_raw_batch(rec.buf.numpy()[:rec.value_len]), now + k, token=k, presence=False)]
                res_keep = rec
            else:
                rg = g.step(raw, off, now + k, presence=False)
                res.append((k, g.encode_block(now + k, rg, boot=0x5eed), None))
        if framed:
            res += [(9, r.block.copy(), None) for _, r in g.drain_framed()]
        print("filter", filt, "framed", framed, [nalt(np.ascontiguousarray(b)) for _, b, _ in res], flush=True)
        del g
        import torch; torch.cuda.empty_cache()
