"""The C-ABI library loads and exports every symbol include/asg.h declares; ctypes
struct layouts match the C header; argument validation works without a GPU (no compute
calls are made here)."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "asg.h")


def _declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(asg_\w+)\s*\(", src, re.M)))


@pytest.fixture(scope="module")
def L():
    from marl_sap_amd import build, _lib
    build.build()
    return _lib.lib()


def test_exports_every_declared_symbol(L):
    from marl_sap_amd import _lib
    names = _declared()
    assert len(names) >= 19
    assert sorted(_lib.EXPORTS) == names
    nm = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    for n in names:
        assert re.search(rf"\bT {n}$", nm, re.M), n
    assert L.asg_abi_version() == 1


def test_struct_layout_matches_header(tmp_path):
    from marl_sap_amd import _lib
    c = tmp_path / "layout.c"
    c.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "asg.h"\nint main(){printf("%zu %zu %zu %zu %zu %zu\\n",'
                 'sizeof(asg_field), sizeof(asg_batch_view), sizeof(asg_config), offsetof(asg_config, seed),'
                 'offsetof(asg_config, T_trans), offsetof(asg_batch_view, filled));return 0;}\n')
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(c), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True).stdout.split()]
    want = [ctypes.sizeof(_lib.AsgField), ctypes.sizeof(_lib.AsgBatchView), ctypes.sizeof(_lib.AsgConfig),
            _lib.AsgConfig.seed.offset, _lib.AsgConfig.T_trans.offset, _lib.AsgBatchView.filled.offset]
    assert got == want


def test_create_validates_without_gpu(L):
    from marl_sap_amd import _lib
    cfg = _lib.AsgConfig(num_envs=4, n=8, m=4, T=5, L=1, lambda_=0.5)
    h = ctypes.c_void_p()
    rc = L.asg_create(ctypes.byref(cfg), 0, None, ctypes.byref(h))
    assert rc == _lib.ASG_E_INVALID_ARG and not h.value
    assert "larger sample" in _lib.last_error()
    with pytest.raises(ValueError, match="larger sample"):
        _lib.check(rc)
    cfg = _lib.AsgConfig(num_envs=0, n=4, m=4, T=5, L=1)
    assert L.asg_create(ctypes.byref(cfg), 0, None, ctypes.byref(h)) == _lib.ASG_E_INVALID_ARG
    cfg = _lib.AsgConfig(num_envs=1, n=4, m=4, T=5, L=1, rng_mode=1, benefit_mode=1)
    assert L.asg_create(ctypes.byref(cfg), 0, None, ctypes.byref(h)) == _lib.ASG_E_INVALID_ARG
    assert "dense" in _lib.last_error()


def test_kernel_entry_points_validate_without_gpu(L):
    from marl_sap_amd import _lib
    st = _lib.i64arr([16, 4, 1])
    assert L.asg_lsa_batched(None, 5, st, 1, 4, 4, 0, None, None, None, None) == _lib.ASG_E_INVALID_ARG
    assert L.asg_lsa_batched(None, 0, st, 1, 2000, 4, 0, None, None, None, None) == _lib.ASG_E_INVALID_ARG
    assert L.asg_lsa_batched(None, 0, st, 0, 4, 4, 0, None, None, None, None) == _lib.ASG_OK  # empty batch
    assert L.asg_haa_select(None, st, None, st, 1, 4, 4, None, 0.5, None, None, None) == _lib.ASG_E_INVALID_ARG
    assert L.asg_epsilon_greedy(None, st, None, st, 1, 4, 4, 0.1, 0, 0, 0, None, st, None, None) == \
        _lib.ASG_E_INVALID_ARG
    assert L.asg_reset(None, None, 0) == _lib.ASG_E_INVALID_ARG
    assert L.asg_step(None, None, 0) == _lib.ASG_E_INVALID_ARG
    assert L.asg_step_ex(None, None, 0, _lib.ASG_STEP_USE_SELECTED_BIDS) == _lib.ASG_E_INVALID_ARG
    assert L.asg_random_rollout(None, None, 0, 20, 1) == _lib.ASG_E_INVALID_ARG
    assert L.asg_bids_select(None, None, None, None, None, 1, 1, 0.1, 0, 1, None) == _lib.ASG_E_INVALID_ARG
    agent = [None] * 5 + [256, 64, 1, None, 0, None, 0.05, 0, 1, None, None]
    assert L.asg_rollout(None, None, 0, 1, 1, 0, *agent) == _lib.ASG_E_INVALID_ARG
    assert L.asg_reset_rollout(None, None, 0, 1, 0, *agent) == _lib.ASG_E_INVALID_ARG
    # asg_filtered_benefits with generated Gaussian noise: n <= 8188 agents (64 KiB of LDS per
    # workgroup on every CDNA part); rejected before any device call above that
    fake = ctypes.c_void_p(16)
    args = lambda n: (fake, st, fake, 1, n, 8, 4, None, 0.5, None, 0, 0, 0, fake, None)  # noqa: E731
    assert L.asg_filtered_benefits(*args(8189)) == _lib.ASG_E_INVALID_ARG
    assert "8188" in _lib.last_error()


def _h2_geom(K, m):
    """asg_h2.hip:h2_geom restated: NB blocks of P inputs, each padded to a multiple of 32;
    block 0 is the one-hot prefix when the input is m (L + 1) values (m >= 16)."""
    blocked = m >= 16 and K % m == 0 and K // m >= 2
    P, NB = (m, K // m) if blocked else (K, 1)
    Pp = (P + 31) // 32 * 32
    return P, NB, Pp, blocked


def test_agent_pack_layout_without_gpu(L):
    """Host-only sizing of the packed agent buffer.  n_out <= 256 (the split-f16 path, GRU or
    Linear, any K): W1^T of the one-hot prefix (prefix geometry), then the section -- header,
    W1 planes over the block-padded inputs, the recurrent planes (GRU: W_ih + W_hh, 6 gates;
    Linear: 1), W2 planes.  n_out > 256: f32 W1 fragments, the GRU as three bf16 planes, f32 W2,
    W1^T of the one-hot prefix when n_out % 16 == 0, n_out < K and K % 32 == 0."""
    mode = L.asg_rnn_agent_mfma_mode()
    assert mode & 1 == 1
    gru = 3 * 4 * 2 * 3 * 64 if mode & 1 else 4 * 12 * 64
    w1x3 = lambda K: (K // 32) * 4 * 3 * 64 if (mode & 2 and K % 32 == 0) else 0  # noqa: E731
    for K, m, rnn in [(256, 64, 1), (1024, 256, 1), (70, 16, 1), (256, 64, 0), (100, 25, 1), (100, 25, 0),
                      (20, 64, 1), (3, 1, 1), (490, 11, 0)]:
        P, NB, Pp, blocked = _h2_geom(K, m)
        size = (16 * P if blocked else 0) + 1 + (Pp * NB // 32) * 512 + (6 if rnn else 1) * 1024 + \
            ((m + 15) // 16) * 256
        assert L.asg_rnn_agent_packed_size(K, 64, m, rnn) == 16 * size, (K, m, rnn)
        assert L.asg_rnn_agent_mode(K, 64, m, rnn) == 4
    for K, m, rnn in [(490, 450, 1), (576, 300, 0)]:
        wr = 2 * gru if rnn else 4 * 4 * 64
        w1 = ((K + 15) // 16) * 4 * 64
        w2 = 4 * ((m + 15) // 16) * 64
        P = m if (m % 16 == 0 and m < K and K % 32 == 0) else 0
        assert L.asg_rnn_agent_packed_size(K, 64, m, rnn) == 16 * (w1 + wr + w2 + 16 * P + w1x3(K)), (K, m, rnn)
        assert L.asg_rnn_agent_mode(K, 64, m, rnn) == mode
    assert L.asg_rnn_agent_packed_size(256, 32, 64, 1) < 0  # hidden must be 64


def test_rollout_l2_slices_without_gpu(L):
    """The fused rollout's LDS plan (asg_rollout_l2_slices): fc1 slices read through L2, -1 for
    shapes asg_rollout rejects (m < 16 or > 256, n > 256, L = 0)."""
    assert L.asg_step_select_l2_slices(64, 64, 3) == L.asg_rollout_l2_slices(64, 64, 3, 1) == 1
    assert L.asg_rollout_l2_slices(64, 64, 3, 0) == 0      # Linear agent: every slice in LDS
    assert L.asg_rollout_l2_slices(64, 64, 1, 1) == 0
    assert L.asg_rollout_l2_slices(256, 256, 3, 1) > 1
    assert L.asg_rollout_l2_slices(20, 25, 3, 1) == 0      # the reference's default shape
    assert L.asg_rollout_l2_slices(30, 64, 3, 1) >= 0
    assert L.asg_rollout_l2_slices(64, 48, 3, 0) >= 0
    assert L.asg_rollout_l2_slices(8, 8, 3, 1) == -1
    assert L.asg_rollout_l2_slices(64, 512, 3, 1) == -1
    assert L.asg_rollout_l2_slices(300, 300, 3, 1) == -1
    assert L.asg_rollout_l2_slices(64, 64, 0, 1) == -1
