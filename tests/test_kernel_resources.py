"""Build-time invariant of the kernels that issue MFMAs from inline asm (csrc/hgemm.hip, csrc/probe.hip): they must
compile without register spills.  hipcc's hazard recognizer does not see an asm MFMA, so a spill the allocator
placed between the last MFMAs and the hand-written wait-state pad would read accumulators before they are written
(the HG_I8_I32 form did: wrong int32 at ragged shapes).  CPU-only: hipcc cross-compiles for gfx950 here."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "bitsandbytes-sycl_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.fixture(scope="module")
def hgemm_device_asm(tmp_path_factory):
    """hgemm.hip compiled ONCE for the module (device code only, ~5 min): its ISA text and the resource-usage remarks."""
    if not os.path.exists(HIPCC):
        pytest.skip("no hipcc")
    s = tmp_path_factory.mktemp("hgemm") / "k.s"
    r = subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                        "-ffp-contract=off", "-I", CSRC, os.path.join(CSRC, "hgemm.hip"), "-o", str(s),
                        "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-2000:]
    return s.read_text(), r.stderr


def _spills(remarks, kernel):
    names, spills = [], []
    for line in remarks.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            names.append(m.group(1))
        m = re.search(r"VGPRs Spill: (\d+)", line)
        if m and names and kernel in names[-1]:
            spills.append((names[-1], int(m.group(1))))
    return spills


def test_hgemm_compiles_spill_free(hgemm_device_asm):
    spills = _spills(hgemm_device_asm[1], "k_hgemm")
    assert spills, "no kernels found"
    assert all(n == 0 for _, n in spills), spills


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="no hipcc")
def test_probe_compiles_spill_free(tmp_path):
    r = subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                        "-ffp-contract=off", "-I", CSRC, os.path.join(CSRC, "probe.hip"), "-o", str(tmp_path / "p.s"),
                        "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    spills = _spills(r.stderr, "k_probe_mfma")
    assert spills, "no kernels found"
    assert all(n == 0 for _, n in spills), spills


def test_hgemm_m0_written_only_by_its_dma_statements(hgemm_device_asm):
    """k_hgemm keeps the LDS-DMA destination in M0 across statements (glds16_chain: one s_add per piece).  That is
    only valid while nothing else in the kernel writes M0: every M0 write in its ISA must be one of the kernel's own
    forms (s_mov_b32 m0, sN / s_add_u32 m0, m0, imm), and no compiler-inserted M0 save or use may appear."""
    text = hgemm_device_asm[0]
    bodies = re.findall(r"^(_ZN3bnb7k_hgemm\w+):[^\n]*\n(.*?)^\.Lfunc_end", text, re.S | re.M)
    assert bodies, "no k_hgemm kernels"
    for name, body in bodies:
        for line in body.splitlines():
            ins = line.split(";")[0].strip()
            if re.search(r"\bm0\b", ins):
                assert re.fullmatch(r"s_mov_b32 m0, s\d+|s_add_u32 m0, m0, (0x[0-9a-f]+|\d+)", ins), (name, ins)


def test_hgemm_tile3_dma_count_between_waits(hgemm_device_asm):
    """The three-barrier k_hgemm schedule (V & 8192) waits `s_waitcnt vmcnt(VM)` once per k-tile, meaning "tile t+1's
    LDS-DMA pieces (issued one k-tile earlier) have landed; the VM issued since may still fly" (256 x 256 tile: 16 pieces,
    VM 13; 256 x 128: 12, 9; 128 x 256: 12, 10; 128 x 128: 8, 6).  That count is only right if exactly `pieces` LDS-DMA instructions --
    and no other vector-memory instruction -- sit between two consecutive waits of the steady-state loop, VM of them
    after the k-tile's first barrier.  Checked on the ISA of every launched kind and tile shape (a miscount would let
    fragment reads see a stage before its DMA landed)."""
    text = hgemm_device_asm[0]
    bodies = re.findall(r"^(_ZN3bnb7k_hgemmILi\dELi(?:8208|40976|106512|237584)\w+):[^\n]*\n(.*?)^\.Lfunc_end", text,
                        re.S | re.M)
    # (40976 = 8208 | HG_V_CWT: the same loop, C stored write-through; 106512 = 40976 | HG_V_EPI: and the interleaved
    # epilogue -- the launched kinds; 237584 = 106512 | HG_V_CNT: the lab's non-temporal C arm)
    assert any("ELi40976E" in b[0] for b in bodies), "no write-through-C k_hgemm kernels"
    assert any("ELi106512E" in b[0] for b in bodies), "no interleaved-epilogue k_hgemm kernels"
    assert bodies, "no three-barrier k_hgemm kernels"
    vmem = re.compile(r"^\s*(global_|buffer_|flat_|scratch_)")
    # per tile shape (WI, WJ): LDS-DMA pieces per k-tile and the vmcnt of barrier B3 (HgPlan3 in hgemm.hip)
    plans = {(8, 8): (16, 13), (8, 4): (12, 9), (4, 8): (12, 10), (4, 4): (8, 6)}
    shapes_seen = set()
    side_seen = False
    for name, body in bodies:
        m = re.search(r"ELb[01]ELi(\d)ELi(\d)E", name)
        assert m, name
        shape = (int(m.group(1)), int(m.group(2)))
        side = re.search(r"ELi\dELi\dELb1EE", name) is not None        # the side-dequantise (prefetch) form
        sides = 0
        shapes_seen.add(shape)
        pieces, vm = plans[shape]
        lines = [ln.split(";")[0].strip() for ln in body.splitlines()]
        # (the side form waits vmcnt(VM + 3) instead when the previous k-tile issued side loads: they may stay in flight)
        # (the prologue's wait for tile 0, vmcnt(WI + WJ), comes before the first barrier: not a B3 wait)
        first_bar = lines.index("s_barrier")
        waits = [i for i, ln in enumerate(lines) if i > first_bar and
                 (ln == f"s_waitcnt vmcnt({vm})" or (side and ln == f"s_waitcnt vmcnt({vm + 3})"))]
        assert len(waits) >= 2, (name, len(waits))
        # the steady-state loop body: consecutive waits inside one basic-block chain (the loop) hold 16 pieces
        counted = 0
        for a, b in zip(waits[:-1], waits[1:]):
            seg = lines[a + 1:b]
            if any(re.match(r"^\.LBB", ln) for ln in seg if ln.endswith(":")) and b - a > 4000:
                continue                                         # first / last tile forms are separate code
            if side and b - a < 16 and not any(vmem.match(ln) for ln in seg):
                continue                                         # the two arms of one B3 wait
            # (the side dequantise's 16-B packed-weight load is one asm statement "s_mov_b32 m0, sN; s_nop 0; load";
            # the GEMM's pieces in the loop are chained "load; s_add_u32 m0, m0, imm")
            code = [j for j, ln in enumerate(seg) if ln]

            def side_x4(i):
                k = code.index(i)
                return k >= 2 and seg[code[k - 1]] == "s_nop 0" and seg[code[k - 2]].startswith("s_mov_b32 m0")
            dma = sum(1 for i, ln in enumerate(seg) if ln.startswith("global_load_lds_dwordx4") and not side_x4(i))
            other = [i for i, ln in enumerate(seg) if vmem.match(ln) and
                     (not ln.startswith("global_load_lds_dwordx4") or side_x4(i))]
            bars = [i for i, ln in enumerate(seg) if ln == "s_barrier"]
            assert len(bars) >= 2, (name, bars)
            if side:
                # the side dequantise's loads / stores: only in the previous k-tile's tail, after its B3 and before this
                # k-tile's B1 (so older than every piece the wait leaves in flight), and only the side's own kinds
                assert all(bars[0] < i < bars[1] for i in other), (name, [seg[i] for i in other][:4])
                assert all(re.match(r"global_(load_lds_dword |load_lds_dwordx4 |load_lds_ubyte |store_dwordx4 )",
                                    seg[i] + " ") for i in other), (name, [seg[i] for i in other][:4])
                sides += bool(other)
                other = []
            assert dma == pieces and not other, (name, dma, [seg[i] for i in other][:3])
            counted += 1
            # of those 16: the previous k-tile's last 3 A pieces (after its barrier B3), then this k-tile's 13 (from its
            # barrier B1 on) before the wait -- the 13 the wait leaves in flight
            before_b1 = sum(1 for i, ln in enumerate(seg[:bars[1]]) if ln.startswith("global_load_lds_dwordx4")
                            and not side_x4(i))
            after_b1 = sum(1 for i, ln in enumerate(seg) if i >= bars[1] and ln.startswith("global_load_lds_dwordx4")
                           and not side_x4(i))
            assert (before_b1, after_b1) == (pieces - vm, vm), (name, before_b1, after_b1)
        assert counted >= 1, name
        assert not side or sides >= 1, name          # (the side form's loop does hold side operations)
        side_seen |= side
    assert shapes_seen == set(plans), shapes_seen
    assert side_seen


def test_hgemm_no_accumulator_copies_between_mfmas(hgemm_device_asm):
    """k_hgemm issues its MFMAs from inline asm with the accumulators pinned to AGPRs ("+a").  hipcc cannot see that such
    a statement is an MFMA, so it inserts no MFMA -> AGPR-read wait states: any v_accvgpr_read / _write / _mov the
    register allocator places between two asm MFMAs may read an accumulator before the MFMA wrote it.  That is what made
    the removed round-3 schedule arm non-deterministic on int8 (192-208 such copies in its loop).  Every
    k_hgemm kernel built into the library must hold none between its first and last MFMA (the epilogue reads the
    accumulators after the hand-written wait-state pad that follows the last one)."""
    text = hgemm_device_asm[0]
    bodies = re.findall(r"^(_ZN3bnb7k_hgemm\w+):[^\n]*\n(.*?)^\.Lfunc_end", text, re.S | re.M)
    assert bodies, "no k_hgemm kernels"
    for name, body in bodies:
        lines = [ln.split(";")[0].strip() for ln in body.splitlines()]
        mf = [i for i, ln in enumerate(lines) if ln.startswith("v_mfma")]
        assert mf, name
        copies = [ln for ln in lines[mf[0]:mf[-1]] if re.match(r"v_accvgpr_(read|write|mov)", ln)]
        assert not copies, (name, len(copies), copies[:3])
