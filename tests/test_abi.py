"""C-ABI library checks that need no GPU: it loads, exports every symbol the
public header declares, and rejects bad arguments on the host before any
launch (SURVEY.md 8(b) error conventions)."""
import ctypes
import os
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent


def test_library_exports_header_symbols(trk):
    L = trk.lib()
    syms = trk.header_symbols()
    assert len(syms) >= 7
    for s in syms:
        assert hasattr(L, s), f"libtrk_amd.so does not export {s}"
    assert L.trk_abi_version() == 2


def test_host_side_argument_errors(trk):
    L = trk.lib()
    # bad input shape -> TRK_EINVAL with a message; no device pointer touched
    rc = L.trk_roi_align_fwd(None, 0, 512, 40, 40, 0, None, 4, 1.0, 7, 7, 2, 1, None, 0, 0, None, 0, None)
    assert rc == -1 and b"bad input shape" in L.trk_last_error()
    rc = L.trk_roi_align_fwd(None, 1, 512, 40, 40, 0, None, 4, 1.0, 7, 7, 0, 1, ctypes.c_void_p(8),
                             0, 0, ctypes.c_void_p(8), 1 << 30, None)
    assert rc == -1  # null input pointer with K > 0
    p = trk.default_cost_params()
    rc = L.trk_build_cost(1, 4, 4, None, None, None, 2000, None, None, None, None, None, None, None,
                          None, None, None, ctypes.byref(p), None, None, None, None, None, None)
    assert rc == -1 and b"Tmax" in L.trk_last_error()  # hist_max above 1024
    nr = (ctypes.c_int32 * 1)(5000)
    nc = (ctypes.c_int32 * 1)(5)
    rc = L.trk_lsap(1, ctypes.c_void_p(8), 0, 5, 25000, nr, nc, 5, ctypes.c_void_p(8), ctypes.c_void_p(8),
                    ctypes.c_void_p(8), ctypes.c_void_p(8), None, 0, 0.0, None)
    assert rc == -1 and b"outside" in L.trk_last_error()
    # empty problems are valid no-ops
    assert L.trk_lsap(0, None, 0, 0, 0, None, None, 0, None, None, None, None, None, 0, 0.0, None) == 0


def test_python_wrappers_reject_host_tensors(trk):
    import torch
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        trk.roi_align(torch.zeros(1, 4, 8, 8), torch.zeros(1, 5), (2, 2), 1.0, 2, True)


def test_encoder_state_dict_keys_and_strict_load(trk):
    import torch
    import gen_common as G
    m = trk.Model(in_channels=512, out_channels=512, warmup_epochs=10, proj_dim=128)
    keys = [k for k, _ in G.encoder_param_shapes()]
    assert list(m.state_dict().keys()) == keys
    assert sum(p.numel() for p in m.parameters()) == 2061570
    sd = {k: torch.from_numpy(v) for k, v in G.seeded_state_dict_np(0).items()}
    m.load_state_dict(sd, strict=True)


@pytest.mark.parametrize("s", [7, 10])
def test_encoder_fused_graph_fp32_vs_reference_golden(trk, s):
    """The fused encoder graph (encoder.py) is pure PyTorch: its fp32 numerics
    are checked here on CPU and again on the GPU in test_gpu_kernels.py."""
    import os
    import torch
    import gen_common as G
    from conftest import GOLDEN
    d = np.load(os.path.join(GOLDEN, "encoder_golden.npz"))
    m = trk.Model(512, 512, 10, 128).eval()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in G.seeded_state_dict_np(0).items()})
    x = torch.from_numpy(G.encoder_input(int(d[f"seed_s{s}"]), 16, s))
    with torch.no_grad():
        z = m(x).numpy()
    assert np.max(np.abs(z - d[f"z_s{s}"])) < 1e-5


def test_rmb_front_fragment_packing_and_argument_errors(trk):
    """enc_pack_fragments is the exact permutation trk_enc_rmb_front_means reads (element
    (g, s, n, l, j) = W[g*512 + 16n + l%16][32s + 8(l//16) + j]); the entry point rejects
    M % 100 != 0 and null pointers on the host."""
    import torch
    from importlib import import_module
    ops = import_module("a-lightweight-unsupervised-feature-extractor-_amd.ops")
    W = torch.arange(1024 * 512, dtype=torch.int64).view(1024, 512)
    P = ops.enc_pack_fragments(W).view(2, 16, 32, 64, 8)
    g, s, n, l, j = torch.meshgrid(*[torch.arange(k) for k in (2, 16, 32, 64, 8)], indexing="ij")
    ref = W[g * 512 + 16 * n + l % 16, 32 * s + 8 * (l // 16) + j]
    assert torch.equal(P, ref)
    assert torch.equal(ops.enc_pack_fragments(W.view(2, 512, 512)), ops.enc_pack_fragments(W))
    L = trk.lib()
    v = ctypes.c_void_p(16)
    assert L.trk_enc_rmb_front_means(None, 0, *([None] * 9)) == 0
    assert L.trk_enc_rmb_front_means(v, 150, *([v] * 9)) == -1
    assert b"M % 100" in L.trk_last_error()
    assert L.trk_enc_rmb_front_means(v, 100, *([v] * 5), None, v, None, v) == -1
    # trk_enc_transition_gemm2: packed weights only for K = 1024, N = 512, kscale = 512
    assert L.trk_enc_transition_gemm2(v, 100, 100, 1024, v, 512, v, v, v, 768, v, None) == -1
    assert b"N = 512" in L.trk_last_error()
    assert L.trk_enc_transition_gemm2(v, 100, 100, 768, v, 512, v, v, v, 512, v, None) == -1
    assert L.trk_enc_se_means(None, 0, 512, None, None, 128, None, None, None, None) == 0
    assert L.trk_enc_se_means(v, 4, 512, v, v, 120, v, v, v, v) == -1
    assert b"multiples of 16" in L.trk_last_error()


def test_no_device_allocation_in_the_library():
    """include/trk_amd.h promises no malloc / free inside a call (calls never synchronise the
    device and are hipGraph-capturable): no HIP allocation, free or memset anywhere in csrc/."""
    import re
    src = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                       "a-lightweight-unsupervised-feature-extractor-_amd", "csrc")
    bad = []
    for name in sorted(os.listdir(src)):
        if name.endswith((".hip", ".cpp", ".h")):
            with open(os.path.join(src, name)) as fh:
                for i, line in enumerate(fh, 1):
                    if re.search(r"\bhip(Malloc\w*|Free\w*|Memset\w*|HostAlloc|HostMalloc)\s*\(", line):
                        bad.append(f"{name}:{i}: {line.strip()}")
    assert not bad, bad


def test_enc_pack_rows_layout(trk):
    """the tail kernels' weight operand order (include/trk_amd.h, "Weight layout"): element
    [t][kb][16 g + r][e] of the packed [N/16][K/16][64][4] is W[16 t + r][16 kb + 4 g + e]"""
    from importlib import import_module
    import torch
    ops = import_module("a-lightweight-unsupervised-feature-extractor-_amd.ops")
    W = torch.randn(48, 64, generator=torch.Generator().manual_seed(3))
    Wp = ops.enc_pack_rows(W)
    assert tuple(Wp.shape) == (3, 4, 64, 4)
    for t, kb, g, r, e in ((0, 0, 0, 0, 0), (2, 3, 3, 15, 3), (1, 2, 1, 7, 2)):
        assert Wp[t, kb, 16 * g + r, e].item() == W[16 * t + r, 16 * kb + 4 * g + e].item()
    assert torch.equal(Wp.reshape(-1).sort().values, W.reshape(-1).sort().values)  # a permutation
    with pytest.raises(ValueError):
        ops.enc_pack_rows(torch.zeros(20, 64))


def test_no_mutable_device_pointer_globals_in_csrc():
    """The library keeps no caller-owned device pointer between calls (r05 verdict: the front's
    progress counter was a process-global; it is now an argument of the launch).  The only
    pointer-holding globals are the trk_*_set_prof diagnostics buffers, and those are
    trk::DiagBuf (bound to the device current when set, handed only to launches on that
    device).  Scans every namespace-scope declaration in csrc/ for a pointer type."""
    import re
    csrc = ROOT / "a-lightweight-unsupervised-feature-extractor-_amd" / "csrc"
    bad, diag = [], []
    for f in sorted(list(csrc.glob("*.hip")) + list(csrc.glob("*.cpp")) + list(csrc.glob("*.h"))):
        depth = 0
        for ln, line in enumerate(f.read_text().splitlines(), 1):
            code = line.split("//")[0]
            at_file_scope = depth == 0 or (depth == 1 and re.match(r"^\S", line) is not None)
            if at_file_scope and re.match(r"^(static\s+)?(const\s+)?[A-Za-z_][\w:<>]*\s*\*+\s*g_\w+\s*(=|;)", code):
                bad.append(f"{f.name}:{ln}: {line.strip()}")
            if re.match(r"^trk::DiagBuf\s+g_\w+;", code):
                diag.append(f.name)
            depth += code.count("{") - code.count("}")
    assert not bad, bad
    assert sorted(diag) == ["cost.hip", "enc_gemm.hip", "enc_head.hip", "lsap.hip"]
    src = (csrc / "enc_gemm.hip").read_text()
    assert "g_rf_progress" not in src and "set_progress" not in src
    assert "(int32_t)(__builtin_amdgcn_readfirstlane(v) - target) >= 0" in src  # wrap-safe gate


def test_buffer_descriptor_bases_zero_extend_their_halves():
    """`__builtin_amdgcn_readfirstlane` returns int: an address half ORed or shifted straight from
    it sign-extends, so a buffer descriptor built that way gets an upper address half of all ones
    whenever bit 31 of the lower half is set (an illegal-address fault that depends on where the
    allocator put the buffer; r06's cost3 fragment image hit it).  Every make_buffer_rsrc base
    must be assembled from uint32_t variables, with no readfirstlane inside the call."""
    import re
    csrc = ROOT / "a-lightweight-unsupervised-feature-extractor-_amd" / "csrc"
    calls = 0
    for f in sorted(csrc.glob("*.hip")):
        src = f.read_text()
        start = 0
        while (k := src.find("__builtin_amdgcn_make_buffer_rsrc(", start)) >= 0:
            i, depth = k + len("__builtin_amdgcn_make_buffer_rsrc("), 1
            while depth:
                depth += {"(": 1, ")": -1}.get(src[i], 0)
                i += 1
            call = src[k:i]
            first = re.split(r",\s*0\s*,", call[len("__builtin_amdgcn_make_buffer_rsrc("):])[0]
            assert "readfirstlane" not in first, f"{f.name}: {call}"
            calls += 1
            start = i
    assert calls >= 4


def test_encoder_odd_sizes_forward_on_cpu(trk, oracle):
    """A Model whose SE hidden size (out_channels / 4 = 10) and proj_dim (24) are not
    multiples of 16 still runs forward (r05 advisor: the tail kernels' weight packing used to
    raise for every forward, including the CPU / fp32 paths that never read it); the packs are
    made only when the fused tail can run.  Checked against the oracle's fp32 eval graph."""
    import torch
    torch.manual_seed(3)
    m = trk.Model(in_channels=48, out_channels=40, warmup_epochs=10, proj_dim=24).eval()
    with torch.no_grad():
        for p in m.parameters():
            p.normal_(0, 0.2)
        for mod in m.modules():
            if isinstance(mod, torch.nn.BatchNorm2d):
                mod.running_mean.normal_(0, 0.1)
                mod.running_var.uniform_(0.5, 1.5)
        x = torch.randn(3, 48, 10, 10)
        z = m(x)
        assert "se_w1_pk" not in m._fused
        ref = oracle.encoder_forward({k: v.float() for k, v in m.state_dict().items()}, x)
    assert z.shape == (3, 24)
    assert (z - ref).abs().max().item() < 1e-5
