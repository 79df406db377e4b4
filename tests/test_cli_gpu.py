"""The file-compatible ldpc CLI and ldpc_amd.decode_files on the GPU (the
ldpc.exe contract, DNA_main.cpp:300-505, 916-927, 965-1182)."""
import os
import shutil
import subprocess

import numpy as np
import pytest

import synth
from conftest import PCHK, ROOT

pytestmark = pytest.mark.gpu
EXE = os.path.join(ROOT, "dna-ldpc-codes_amd", "bin", "ldpc")


def _write_inputs(d, codeword, llr, i=1):
    cwb = f"codeword_n18432_m1860_{i}"
    soft = f"soft72000_n18432_m1860_{i}"
    with open(os.path.join(d, cwb + ".txt"), "w") as f:  # def_func.write_codeword format
        f.write("".join(f"{int(b)} " for b in codeword))
    with open(os.path.join(d, soft + ".txt"), "w") as f:  # str(float) as decoder.py:533
        f.write("".join(str(float(v)) + " " for v in llr))
    shutil.copyfile(PCHK, os.path.join(d, "decode_n18432_m2048_final.pchk"))
    return cwb, soft


@pytest.mark.parametrize("algo,dtype", [("bp", 0), ("msa", 20)])
def test_cli_matches_oracle(tmp_path, og, codewords, algo, dtype):
    d = str(tmp_path)
    llr = synth.dna_like_llrs(codewords, seed=1, reads=57000)[13]  # codeword 14: a BP failure case
    if algo == "msa":
        llr = synth.bsc_llrs(codewords, 0, 1, seed=2026, p=0.002)[0]
    cwb, soft = _write_inputs(d, codewords[13] if algo == "bp" else codewords[0], llr)
    argv = [EXE, "0", str(dtype), "0", "7", "200", "1", cwb, soft, "decode_n18432_m2048_final", "0", "0", "0", "0"]
    r = subprocess.run(argv, cwd=d, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "g_CODE_N : 18432" in r.stdout and f"dec_{cwb}.txt" in r.stdout
    dec = np.array(open(os.path.join(d, f"dec_{cwb}.txt")).read().split(), dtype=np.uint8)
    h, _, it, v = og.decode_batch(llr[None, :], 200, algo=0 if algo == "bp" else 1, threads=1, want_post=False)
    assert np.array_equal(dec, h[0])
    res = os.path.join(d, f"result_({soft}.txt)_decode_n18432_m2048_final.pchk_{dtype}_0.000dB_0_200_7.txt")
    txt = open(res).read()
    assert "dv            : 8" in txt and "dc            : 72" in txt and "bRegular_dc   : 1" in txt
    truth = codewords[13] if algo == "bp" else codewords[0]
    nerr = int((h[0] != truth).sum())
    assert f"# of Bit Errors[ 1]     : {nerr}" in txt
    raw = int((truth != (llr < 0)).sum())
    assert f"# of Bit Errors[ 0]     : {raw}" in txt


def test_decode_files_matches_cli(tmp_path, codewords, gpu):
    d = str(tmp_path)
    llr = synth.dna_like_llrs(codewords, seed=0)[4]
    cwb, soft = _write_inputs(d, codewords[4], llr, i=5)
    out = gpu.decode_files(cwb, soft, "decode_n18432_m2048_final", max_iter=200, directory=d)
    assert out["bit_errors"] == 0 and out["valid"]
    py_dec = open(os.path.join(d, out["dec_file"])).read()
    os.remove(os.path.join(d, out["dec_file"]))
    subprocess.run([EXE, "0", "0", "0", "7", "200", "1", cwb, soft, "decode_n18432_m2048_final", "0", "0", "0", "0"],
                   cwd=d, check=True, capture_output=True, timeout=120)
    assert open(os.path.join(d, out["dec_file"])).read() == py_dec


def test_cli_targeting_and_frames(tmp_path, codewords):
    d = str(tmp_path)
    llr = synth.bsc_llrs(codewords, 0, 1, seed=1, p=0.02)[0]
    cwb, soft = _write_inputs(d, codewords[0], llr)
    argv = [EXE, "0", "0", "0", "7", "5", "3", cwb, soft, "decode_n18432_m2048_final", "0", "0", "0", "1", "1", "100"]
    r = subprocess.run(argv, cwd=d, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    res = os.path.join(d, f"result_({soft}.txt)_decode_n18432_m2048_final.pchk_0_0.000dB_0_5_7.txt")
    txt = open(res).read()
    assert "target_VN:1~100" in txt and "# of Frame[ 0]          :3" in txt


def test_config1_plumbing_cli(tmp_path, og, codewords):
    """B = 1, codeword_n18432_m1860_1, LLR +-ln 49 from
    BSC p = 0.02 drawn with numpy default_rng(0), 50 BP iterations through the
    file-compatible CLI; the decode fails after all 50 iterations, as in the
    oracle."""
    d = str(tmp_path)
    rng = np.random.default_rng(0)
    y = codewords[0] ^ (rng.random(codewords.shape[1]) < 0.02).astype(np.uint8)
    llr = np.where(y == 1, -synth.LLR_UNIT, synth.LLR_UNIT)
    cwb, soft = _write_inputs(d, codewords[0], llr)
    argv = [EXE, "0", "0", "0", "7", "50", "1", cwb, soft, "decode_n18432_m2048_final", "0", "0", "0", "0"]
    r = subprocess.run(argv, cwd=d, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    dec = np.array(open(os.path.join(d, f"dec_{cwb}.txt")).read().split(), dtype=np.uint8)
    h, _, it, v = og.decode_batch(llr[None, :], 50, algo=0, threads=1, want_post=False)
    assert it[0] == 50 and not v[0]
    assert np.array_equal(dec, h[0])


@pytest.mark.parametrize("dtype,algo", [(1, 3), (2, 4), (3, 5), (21, 1), (22, 1)])
def test_cli_other_decoder_types(tmp_path, og, codewords, dtype, algo):
    """decoder_type 1/2/3 -> Gallager A/B1/B2 on the soft input's hard
    decision, 21/22 -> float min-sum (the DNA build's g_precision = 0)."""
    d = str(tmp_path)
    llr = synth.bsc_llrs(codewords, 0, 1, seed=99, p=0.002)[0]
    cwb, soft = _write_inputs(d, codewords[0], llr)
    argv = [EXE, "0", str(dtype), "0", "7", "30", "1", cwb, soft, "decode_n18432_m2048_final", "0", "0", "0", "0"]
    r = subprocess.run(argv, cwd=d, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    dec = np.array(open(os.path.join(d, f"dec_{cwb}.txt")).read().split(), dtype=np.uint8)
    if algo == 1:
        h, _, _, _ = og.decode_batch(llr[None, :], 30, algo=1, threads=1, want_post=False)
    else:
        h, _, _, _ = og.decode_int_batch(llr[None, :], 30, algo)
    assert np.array_equal(dec, h[0])


def _cli(d, dtype, cwb, soft, max_iter, tail, channel="0", param="0"):
    argv = [EXE, "0", str(dtype), channel, "7", str(max_iter), "1", cwb, soft, "decode_n18432_m2048_final", param,
            *map(str, tail)]
    r = subprocess.run(argv, cwd=d, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    return np.array(open(os.path.join(d, f"dec_{cwb}.txt")).read().split(), dtype=np.uint8)


def test_cli_puncturing_shortening(tmp_path, og, codewords):
    """LDPC_Channel (DNA_main.cpp:1375-1441): puncturing type 1 sets LR = 1
    on bits start..end (AWGN and BSC), shortening type 1 sets LR = exp(30) (AWGN);
    BP decodes the edited LR, min-sum the unedited LLR.  Type 2 punctures
    start..end of every SC position, stepping by <pchk>.txt's multiplicities.
    Result file: code rate of Set_Code (:574-597) and the type lines."""
    d = str(tmp_path)
    llr = synth.dna_like_llrs(codewords, seed=1, reads=58000)[20]
    cwb, soft = _write_inputs(d, codewords[20], llr)

    def ref(x, algo=0, it=60):
        return og.decode_batch(x[None, :], it, algo=algo, threads=1, want_post=False)[0][0]

    def edited(tail, x, **kw):
        # max_iter 0 returns the initial decisions: the edit must show there
        h0 = _cli(d, 0, cwb, soft, 0, tail, **kw)
        assert np.array_equal(h0, ref(x, it=0)) and not np.array_equal(h0, ref(llr, it=0))
        return _cli(d, 0, cwb, soft, 60, tail, **kw)

    x = llr.copy()
    x[99:400] = 0.0  # bits 100..400
    assert np.array_equal(edited((1, 0, 0, 100, 400), x), ref(x))
    res = os.path.join(d, f"result_({soft}.txt)_decode_n18432_m2048_final.pchk_0_0.000dB_0_60_7.txt")
    txt = open(res).read()
    assert "[Type: 1] Punctuation_VN:100~400 \n\n" in txt
    assert "code rate     : %.3f\n" % (1.0 - (2048 - 301) / (18432 - 301)) in txt
    assert np.array_equal(edited((1, 0, 0, 100, 400), x, channel="1", param="0.02"), ref(x))
    # min-sum reads g_received_LLR, which puncturing leaves alone
    assert np.array_equal(_cli(d, 20, cwb, soft, 60, (1, 0, 0, 100, 400)), ref(llr, algo=1))

    x = llr.copy()
    x[4999:5100] = 30.0
    assert np.array_equal(edited((0, 1, 1, 5000, 5100, 1, 18432), x), ref(x))
    txt = open(res).read()
    assert "target_VN:1~18432 \n\n[Type: 1] Shortening_VN:5000~5100 \n\n" in txt
    assert "code rate     : %.3f\n" % (1.0 - 2048 / (18432 - 101)) in txt
    # BSC: the reference shortens only on AWGN / BEC
    assert np.array_equal(_cli(d, 0, cwb, soft, 0, (0, 1, 0, 5000, 5100), channel="1", param="0.02"), ref(llr, it=0))

    with open(os.path.join(d, "decode_n18432_m2048_final.txt"), "w") as f:
        f.write("".join(f"{m}\n" for m in [256, 512, 1024, 7, 7]))  # M (w + L - 1 = 4 entries), then Mc
    x = llr.copy()
    for base in (0, 256, 768):  # L = 3 positions
        x[base + 9:base + 20] = 0.0  # bits 10..20 of each
    assert np.array_equal(edited((2, 0, 0, 10, 20, 2, 3), x), ref(x))
    txt = open(res).read()
    assert "[Type: 2] Punctuation_VN:10~20 \n\n" in txt
    assert "code rate     : %.3f\n" % (1.0 - (2048 - 33) / (18432 - 33)) in txt


@pytest.mark.parametrize("algo,dtype", [("bp", 0), ("msa", 20)])
def test_cli_nonfinite_tokens(tmp_path, og, codewords, algo, dtype):
    """Soft-file tokens fscanf("%lf") accepts and Python's str() writes for
    non-finite floats -- nan, inf, -inf -- plus an exponent form and a hex
    float: the CLI reads them (cli_io.cpp, strtod) and decodes what the oracle
    decodes on the same values (the NaN / overflow guards of dec.cpp:676-687
    on the device)."""
    d = str(tmp_path)
    llr = synth.bsc_llrs(codewords, 0, 1, seed=11, p=0.002)[0].copy()
    toks = [str(float(v)) for v in llr]
    for j, t in ((5, "nan"), (77, "inf"), (901, "-inf"), (4000, "1e-300"), (4001, "0x1.8p1"), (9000, "-0.0")):
        toks[j] = t
        llr[j] = float.fromhex(t) if t.startswith("0x") else float(t)
    cwb, soft = f"codeword_n18432_m1860_3", f"soft72000_n18432_m1860_3"
    with open(os.path.join(d, cwb + ".txt"), "w") as f:
        f.write("".join(f"{int(b)} " for b in codewords[0]))
    with open(os.path.join(d, soft + ".txt"), "w") as f:
        f.write(" ".join(toks) + "\n")
    shutil.copyfile(PCHK, os.path.join(d, "decode_n18432_m2048_final.pchk"))
    argv = [EXE, "0", str(dtype), "0", "7", "40", "1", cwb, soft, "decode_n18432_m2048_final", "0", "0", "0", "0"]
    r = subprocess.run(argv, cwd=d, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    dec = np.array(open(os.path.join(d, f"dec_{cwb}.txt")).read().split(), dtype=np.uint8)
    h, _, _, _ = og.decode_batch(llr[None, :], 40, algo=0 if algo == "bp" else 1, threads=1, want_post=False)
    assert np.array_equal(dec, h[0])
