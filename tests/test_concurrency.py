"""The C-ABI's threading contract: a loaded graph is immutable
and shareable across threads, calls are reentrant, and ldpc_last_error is
per thread.  The reference keeps all of its state in globals
(rcode.cpp:33-45, dec.cpp:39-83, DNA_main.cpp:145-295), so it has no
equivalent; these pin the replacement's contract."""
import threading

import numpy as np
import pytest

import synth
from conftest import PCHK


def _run_threads(fns):
    out, errs = [None] * len(fns), []
    barrier = threading.Barrier(len(fns))

    def wrap(i, f):
        try:
            barrier.wait()
            out[i] = f()
        except Exception as e:  # noqa: BLE001 -- reported below
            errs.append(e)

    ts = [threading.Thread(target=wrap, args=(i, f)) for i, f in enumerate(fns)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in ts), "thread did not finish"
    if errs:
        raise errs[0]
    return out


def test_concurrent_graph_loads_and_thread_local_errors(L, tmp_path):
    """Eight threads load the DNA code at once and read back identical edge
    lists; threads that fail (missing file, bad magic) see their own error
    code and message while the others succeed."""
    bad = tmp_path / "bad.pchk"
    bad.write_bytes(b"\x00\x01\x02\x03" * 8)
    ref = L.Graph(PCHK).edges()

    def good():
        g = L.Graph(PCHK)
        return [np.array_equal(a, b) for a, b in zip(g.edges(), ref)], (L.lib().ldpc_last_error() or b"")

    def missing():
        with pytest.raises(L.LdpcError) as ei:
            L.Graph(str(tmp_path / "nope.pchk"))
        return ei.value.code, str(ei.value)

    def badmagic():
        with pytest.raises(L.LdpcError) as ei:
            L.Graph(str(bad))
        return ei.value.code, str(ei.value)

    res = _run_threads([good, missing, good, badmagic, good, missing, good, badmagic])
    for i in (0, 2, 4, 6):
        assert all(res[i][0])
    assert res[1][0] == res[5][0] and "nope.pchk" in res[1][1]
    assert res[3][0] == res[7][0] and res[3][0] != res[1][0]


@pytest.mark.gpu
def test_concurrent_decodes_share_one_graph(gpu, codewords):
    """Six threads decode different batches through one graph at once (BP and
    min-sum, with and without posteriors, DNA-batch and host-exp paths);
    every result equals the same call made alone."""
    G = gpu.Graph(PCHK)
    jobs = [
        (synth.dna_like_llrs(codewords, seed=11, reads=58000)[:130], "bp", "llr", 60),
        (synth.bsc_llrs(codewords, 0, 96, seed=7, p=0.003), "bp", None, 40),
        (synth.bsc_llrs(codewords, 96, 80, seed=8, p=0.002), "msa", "llr", 40),
        (synth.dna_like_llrs(codewords, seed=12, reads=60000)[:272], "bp", None, 200),
        (synth.bsc_llrs(codewords, 10, 70, seed=9, p=0.02), "bp", "ratio", 20),
        (synth.bsc_llrs(codewords, 20, 64, seed=10, p=0.004), "msa", None, 30),
    ]
    alone = [G.decode(x, max_iter=it, algo=a, post=p) for x, a, p, it in jobs]
    for _ in range(2):
        together = _run_threads([lambda j=j: G.decode(j[0], max_iter=j[3], algo=j[1], post=j[2]) for j in jobs])
        for (h0, p0, i0, v0), (h1, p1, i1, v1) in zip(alone, together):
            assert np.array_equal(h0, h1) and np.array_equal(i0, i1) and np.array_equal(v0, v1)
            if p0 is not None:
                assert np.array_equal(p0.view(np.uint64), p1.view(np.uint64))
