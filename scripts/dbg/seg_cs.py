"""Debug: which page words does the GPU encoder's page checksum cover? (n-row blocks, GPU vs CPU)"""
import sys
import numpy as np
sys.path.insert(0, ".")
from tests.test_gpu_segments import _encode_gpu
from tests.test_segments import synth_rows
from sitewhere_amd.persistence import segments as sg

M = (1 << 64) - 1


def mix(x):
    x ^= x >> 30; x = (x * 0xbf58476d1ce4e5b9) & M
    x ^= x >> 27; x = (x * 0x94d049bb133111eb) & M
    return x ^ (x >> 31)


def wmix(w, i):
    return mix((w + (i + 1) * 0x9E3779B97F4A7C15) & M)


for n in (1, 3, 1024):
    rows, recs, spans, raw = synth_rows(n, seed=n)
    g = _encode_gpu(rows, recs, spans, raw, seed=n)
    c = sg.encode_block(rows, recs, spans, raw)
    print("n", n, "len", len(g), len(c), "verify gpu", sg.verify(g), "cpu", sg.verify(c),
          "diff bytes", np.nonzero(g != c)[0][:16] if len(g) == len(c) else "len")
    hdr = np.frombuffer(c[:64].tobytes(), sg.HDR)[0]
    np_ = int(hdr["n_pages"])
    po = np.frombuffer(c[64:64 + 4 * (np_ + 1)].tobytes(), np.uint32)
    for p in range(np_):
        for name, b in (("cpu", c), ("gpu", g)):
            pg = b[po[p]:po[p + 1]].tobytes()
            words = np.frombuffer(pg, np.uint64)
            heap_off = int(np.frombuffer(pg[16:20], np.uint32)[0])
            stored = int(words[1])
            contrib = [wmix(int(w), i) for i, w in enumerate(words)]
            def x(idx):
                r = 0
                for i in idx:
                    r ^= contrib[i]
                return r
            allw = [i for i in range(len(words)) if i != 1]
            hyp = {"all": x(allw), "no_heap": x([i for i in allw if i < heap_off // 8]),
                   "hdr_only": x([i for i in allw if i < 50]), "no_hdr": x([i for i in allw if i >= 50])}
            print(" page", p, name, "words", len(words), "heap_off", heap_off, "stored==",
                  [k for k, v in hyp.items() if v == stored] or hex(stored))
            if name == "gpu":
                # single-word omissions / extras
                for i in allw:
                    if (hyp["all"] ^ contrib[i]) == stored:
                        print("   gpu checksum misses word", i)
