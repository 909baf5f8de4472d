"""Debug: GPU vs CPU page headers field by field."""
import sys
import numpy as np
sys.path.insert(0, ".")
from tests.test_gpu_segments import _encode_gpu
from tests.test_segments import synth_rows
from sitewhere_amd.persistence import segments as sg

COL = np.dtype([("base", "<u8"), ("data_off", "<u4"), ("count", "<u2"), ("n_exc", "<u2"), ("bits", "u1"),
                ("exp", "i1"), ("pad", "V6")])
assert COL.itemsize == 24
for n in (1, 3):
    rows, recs, spans, raw = synth_rows(n, seed=n)
    g = _encode_gpu(rows, recs, spans, raw, seed=n)
    c = sg.encode_block(rows, recs, spans, raw)
    print("n", n, "spans", spans, "alt lens", spans["alt_len"] if "alt_len" in spans.dtype.names else None)
    for name, b in (("cpu", c), ("gpu", g)):
        pg = b[72:72 + 400].tobytes()
        cols = np.frombuffer(pg[40:400], COL)
        print(name, "pfx", pg[24], "mode", pg[25], "width", pg[26], "heap", np.frombuffer(pg[16:24], np.uint32))
        for i, cc in enumerate(cols):
            print("   col", i, hex(int(cc["base"])), int(cc["data_off"]), int(cc["count"]), int(cc["n_exc"]),
                  int(cc["bits"]), int(cc["exp"]))
