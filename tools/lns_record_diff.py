"""Which CellRecord bytes differ between the lean N-S path and the split
kernels (debug helper for tests/test_gpu_kernels.py::test_lean_ns_equals_split).
python tools/lns_record_diff.py [resonator|wedge_keps]"""
import sys

import numpy as np

sys.path.insert(0, ".")
import openhyperflow2d_amd as hf  # noqa: E402
from openhyperflow2d_amd.models import decks  # noqa: E402

NAMES = [("S", 0, 72), ("dSdx", 72, 144), ("dSdy", 144, 216), ("TurbType", 216, 224), ("l_min", 224, 232),
         ("y_plus", 232, 240), ("Re_local", 240, 248), ("mu_t", 248, 256), ("lam_t", 256, 264),
         ("dkdx..depsdy", 264, 296), ("x,y,ix,iy,nb", 296, 352), ("p", 352, 360), ("id/NG", 360, 384),
         ("CT", 384, 392), ("wall", 392, 400), ("beta", 400, 472), ("Q_conv", 472, 480), ("time", 480, 488),
         ("k", 488, 496), ("R", 496, 504), ("lam", 504, 512), ("mu", 512, 520), ("CP", 520, 528), ("Diff", 528, 536),
         ("Tf", 536, 544), ("A", 544, 616), ("B", 616, 688), ("F", 688, 760), ("RX", 760, 832), ("RY", 832, 904),
         ("Src", 904, 976), ("SrcAdd", 976, 1048), ("Tg,U,V", 1048, 1072), ("Y", 1072, 1104), ("Uw,Vw", 1104, 1120),
         ("droY", 1120, 1184), ("grad", 1184, 1232), ("BGX,BGY", 1232, 1248)]


def main():
    deck = sys.argv[1] if len(sys.argv) > 1 else "resonator"
    text = (decks.resonator(300, 40, nmax=10 ** 6, nout=10 ** 5) if deck == "resonator" else
            decks.wedge15(200, 60, navier_stokes=True, turbulence=4, nmax=10 ** 6, nout=10 ** 5))
    a = hf.Simulation(text, "gpu")
    b = hf.Simulation(text, "gpu")
    b.solver.lean_ns = False
    a.solver.use_graph = b.solver.use_graph = False
    for n, res in [(4, True), (30, False), (6, True), (19, False)]:
        a.step(n, residual=res)
        b.step(n, residual=res)
    print("lns_ok", a.solver.lns_ok, a.solver.lns_why, "steps", a.solver.lns_steps)
    ra = np.frombuffer(a.records(), dtype=np.uint8).reshape(-1, 1248)
    rb = np.frombuffer(b.records(), dtype=np.uint8).reshape(-1, 1248)
    d = ra != rb
    for name, o0, o1 in NAMES:
        cells = np.nonzero(d[:, o0:o1].any(axis=1))[0]
        if len(cells):
            va = ra[cells[0], o0:o1].view(np.float64) if (o1 - o0) % 8 == 0 else None
            vb = rb[cells[0], o0:o1].view(np.float64) if (o1 - o0) % 8 == 0 else None
            print("%-12s %6d cells differ, first cell %d: %s vs %s" % (name, len(cells), cells[0], va, vb))


if __name__ == "__main__":
    main()
