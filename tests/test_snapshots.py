"""Path snapshots: the tutorials' `append!(paths,
[deepcopy(bb.b.XX)])` (docs/src/tutorials/biblock/smoothing.md:55) kept in HBM and streamed to a
DMTPATH1 file (include/dmt.h).  CPU: the reader against a file built from the documented layout,
and the C header's struct size; GPU: device snapshots == downloads at the same iterations, file
round trip bit for bit."""
import os
import subprocess

import numpy as np
import pytest

from diffusionmcmctools_amd import _lib as L
from diffusionmcmctools_amd import workloads as W
from diffusionmcmctools_amd.engine import SNAPSHOT_HEADER, read_snapshots

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _write_reference_file(path, nseg, npts, t, slots, d, m, mask, grid_shared=0):
    """Writes the layout include/dmt.h documents, independently of libdmt."""
    R, G, P = len(nseg), len(npts), int(np.sum(npts))
    hd = np.zeros(1, dtype=SNAPSHOT_HEADER)
    hd["magic"], hd["version"], hd["what_mask"] = b"DMTPATH1", 1, mask
    hd["d"], hd["m"], hd["grid_shared"], hd["precision"] = d, m, grid_shared, 0
    hd["n_recordings"], hd["n_segments"], hd["n_points"] = R, G, P
    hd["n_t"], hd["n_slots"], hd["seg_base"] = len(t), len(slots), 0
    with open(path, "wb") as f:
        f.write(hd.tobytes())
        f.write(np.asarray(nseg, "<i4").tobytes())
        f.write(np.asarray(npts, "<i4").tobytes())
        f.write(np.asarray(t, "<f8").tobytes())
        for it, unit, X, Wp in slots:
            f.write(np.array([it, unit], "<i8").tobytes())
            if mask & 1:
                f.write(np.ascontiguousarray(X, "<f8").tobytes())
            if mask & 2:
                f.write(np.ascontiguousarray(Wp, "<f8").tobytes())


@pytest.mark.parametrize("mask", [1, 2, 3])
def test_reader_follows_documented_layout(tmp_path, mask):
    rng = np.random.default_rng(0)
    nseg, npts = [2, 1, 3], [5, 7, 4, 3, 6, 2]
    P, d, m = sum(npts), 2, 1
    t = rng.random(P)
    slots = [(400 * (k + 1), k % 2, rng.standard_normal((P, d)), rng.standard_normal((P, m)))
             for k in range(3)]
    f = tmp_path / "paths.dmtp"
    _write_reference_file(f, nseg, npts, t, slots, d, m, mask)
    s = read_snapshots(f)
    assert s["n_points"] == [[5, 7], [4], [3, 6, 2]]
    assert s["n_slots"] == 3 and s["d"] == d and s["m"] == m
    assert np.array_equal(s["t"], t)
    assert s["mcmciter"].tolist() == [400, 800, 1200] and s["unit"].tolist() == [0, 1, 0]
    for k, (_, _, X, Wp) in enumerate(slots):
        if mask & 1:
            assert np.array_equal(s["X"][k], X)
            segs = s["paths"](k, 2)  # recording 2: segments 3, 4, 5
            assert [a.shape for a in segs] == [(3, 2), (6, 2), (2, 2)]
            assert np.array_equal(np.concatenate(segs), X[16:])
        if mask & 2:
            assert np.array_equal(s["W"][k], Wp)


def test_reader_rejects_other_files(tmp_path):
    f = tmp_path / "x.bin"
    f.write_bytes(b"\0" * 200)
    with pytest.raises(ValueError):
        read_snapshots(f)


def test_c_header_struct_matches_reader(tmp_path):
    src = tmp_path / "sz.c"
    src.write_text('#include "dmt.h"\n#include <stdio.h>\n#include <stddef.h>\n'
                   'int main(void){printf("%zu %zu\\n", sizeof(dmt_snapshot_header),'
                   ' offsetof(dmt_snapshot_header, n_recordings)); return 0;}\n')
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)],
                   check=True)
    size, off = map(int, subprocess.run([str(exe)], capture_output=True, text=True,
                                        check=True).stdout.split())
    assert size == SNAPSHOT_HEADER.itemsize == 80
    assert off == SNAPSHOT_HEADER.fields["n_recordings"][1]


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["c2", "ragged"])
def test_device_snapshots_and_file_round_trip(tmp_path, cfg):
    import _cases as cs
    import diffusionmcmctools_amd as d
    if cfg == "c2":
        w = W.c2_ou2d(B=150, N=90)
        w.meta["hist_len"] = 40
        ens = d.Ensemble(w.model.kind, w.d, w.m, w.n_points, precision=w.precision, seed=5,
                         grid_shared=w.grid_shared)
        lay = W.fill(ens, w)
        nb = w.nblocks
        t_expect = w.t
    else:
        case, ens, _, ((lay, nb), _) = cs.ragged_pair(hist_len=40)
        t_expect = case["t"]
    ens.loglikhd(lay, L.U, 0, nb)
    ens.snapshot_reserve(4, what_mask=3)
    ref = []
    for k in range(4):
        ens.mcmc_run(lay, 0, nb, 1 + 8 * k, 8)
        ens.snapshot_take(k, mcmciter=8 * (k + 1))
        ref.append((ens.download_paths(L.U, 0), ens.download_paths(L.U, 1)))
    ens.mcmc_run(lay, 0, nb, 33, 4)  # later iterations leave the slots alone
    for k in range(4):
        X, it = ens.snapshot_download(k, 0)
        Wc, _ = ens.snapshot_download(k, 1)
        assert it == 8 * (k + 1)
        assert np.array_equal(X, ref[k][0]) and np.array_equal(Wc, ref[k][1])
    f = tmp_path / "run.dmtp"
    ens.snapshot_write(f, 1, 4)
    s = read_snapshots(f)
    assert s["n_slots"] == 3 and s["mcmciter"].tolist() == [16, 24, 32]
    assert np.array_equal(s["t"], np.asarray(t_expect, dtype=np.float64)[: s["n_t"]])
    for j, k in enumerate(range(1, 4)):
        assert np.array_equal(s["X"][j], ref[k][0]) and np.array_equal(s["W"][j], ref[k][1])
    ens.close()


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["c2", "ragged"])
def test_snapshots_inside_mcmc_run(cfg):
    """dmt_set_run_snapshots: one mcmc_run of 23 iterations from iteration 3 with every = 5
    snapshots u after iterations 5, 10, 15, 20, 25 into a 4-slot ring (the 5th wraps to slot
    0) — the same paths and results as stopping the run there and downloading u, and the same
    per-iteration fetch_ll values as an unsplit run (auto stream keys)."""
    import _cases as cs
    import diffusionmcmctools_amd as d

    def build():
        if cfg == "c2":
            w = W.c2_ou2d(B=150, N=90)
            w.meta["hist_len"] = 40
            ens = d.Ensemble(w.model.kind, w.d, w.m, w.n_points, precision=w.precision, seed=5,
                             grid_shared=w.grid_shared)
            lay = W.fill(ens, w)
            nb = w.nblocks
        else:
            _, ens, _, ((lay, nb), _) = cs.ragged_pair(hist_len=40)
        ens.loglikhd(lay, L.U, 0, nb)
        return ens, lay, nb
    e0, lay, nb = build()
    e1, _, _ = build()
    e0.snapshot_reserve(4, what_mask=3)
    e0.set_run_snapshots(5, slot0=0)
    r0 = e0.mcmc_run(lay, 0, nb, 3, 23)
    ref, r1 = {}, []
    for a, b in ((3, 5), (6, 10), (11, 15), (16, 20), (21, 25)):
        r1.append(e1.mcmc_run(lay, 0, nb, a, b - a + 1))
        ref[b] = (e1.download_paths(L.U, 0), e1.download_paths(L.U, 1))
    assert np.array_equal(r0, np.concatenate(r1[:5]))
    for slot, it in ((1, 10), (2, 15), (3, 20), (0, 25)):
        X, got_it = e0.snapshot_download(slot, 0)
        Wc, _ = e0.snapshot_download(slot, 1)
        assert got_it == it
        assert np.array_equal(X, ref[it][0]) and np.array_equal(Wc, ref[it][1])
    e0.set_run_snapshots(0)
    e0.close()
    e1.close()
