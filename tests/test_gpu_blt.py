"""blt_mm (csrc/blt_gemm.cpp: hipBLASLt called directly, the fastest of its candidates per shape)
against an fp32 PyTorch reference of the same product, over every operand layout the model
issues: transposed operands passed as storage + flag, row slices with their own leading
dimension, beta = 1 accumulation, fp32 / bf16 bias epilogues, bf16 output."""
import pytest
import torch

from textsummarization_on_flink_amd.models.pointer_generator import gemm
from textsummarization_on_flink_amd.ops import ops
from textsummarization_on_flink_amd.utils.graphs import capture_guard

pytestmark = pytest.mark.gpu

BF, F32 = torch.bfloat16, torch.float32


def _ref(a, b):
    return a.float() @ b.float()


@pytest.mark.parametrize("ta", [False, True])
@pytest.mark.parametrize("tb", [False, True])
@pytest.mark.parametrize("M,N,K", [(96, 80, 64), (1000, 256, 520), (256, 512, 40000)])
def test_blt_layouts_match_fp32(ta, tb, M, N, K):
    g = torch.Generator(device="cuda").manual_seed(M + N + K + 2 * ta + tb)
    r = lambda *s: (torch.randn(*s, device="cuda", generator=g) * 0.1).to(BF)
    a = r(K, M).t() if ta else r(M, K)
    b = r(N, K).t() if tb else r(K, N)
    out = torch.empty(M, N, device="cuda", dtype=F32)
    gemm(out, a, b)
    torch.testing.assert_close(out, _ref(a, b), rtol=2e-3, atol=2e-3 * (K ** 0.5) * 0.01 + 1e-4)


def test_blt_beta_bias_slices_and_bf16_out():
    k = ops()
    g = torch.Generator(device="cuda").manual_seed(7)
    r = lambda *s: (torch.randn(*s, device="cuda", generator=g) * 0.1).to(BF)
    M, N, K = 700, 384, 256
    # row slice of a wider buffer (leading dimension 392 > N) and an operand slice with ld > K
    wide = torch.zeros(M, N + 8, device="cuda", dtype=F32)
    out = wide[:, :N]
    abuf = r(M, K + 8)
    a = abuf[:, :K]
    b = r(K, N)
    bias = torch.randn(N, device="cuda", generator=g)
    gemm(out, a, b, 0.0, bias)
    ref = _ref(a, b) + bias
    torch.testing.assert_close(out, ref, rtol=2e-3, atol=1e-3)
    assert torch.all(wide[:, N:] == 0)  # nothing written past the slice
    # beta = 1 accumulates into the slice
    a2, b2 = r(M, 128), r(N, 128).t()
    gemm(out, a2, b2, 1.0)
    torch.testing.assert_close(out, ref + _ref(a2, b2), rtol=2e-3, atol=1e-3)
    # bf16 output with a bf16 bias epilogue (the logits GEMM)
    ob = torch.empty(M, N, device="cuda", dtype=BF)
    bb = bias.to(BF)
    gemm(ob, a, b, 0.0, bb)
    torch.testing.assert_close(ob.float(), _ref(a, b) + bb.float(), rtol=1e-2, atol=1e-2)
    st = k.blt_stats()
    assert st[0] >= 3 and st[2] >= 3  # keys seen, calls made
    assert st[1] >= 1                 # at least one key tuned (eager calls)


def test_blt_shares_torchs_hipblaslt():
    """One hipBLASLt instance in the process: _C.so's NEEDED entry resolves to the copy torch
    loaded (same SONAME), not a second one from /opt/rocm."""
    ops()
    torch.mm(torch.ones(8, 8, device="cuda", dtype=BF), torch.ones(8, 8, device="cuda", dtype=BF))
    with open("/proc/self/maps") as f:
        libs = {line.split()[-1] for line in f if "libhipblaslt" in line and line.split()[-1].startswith("/")}
    assert len(libs) == 1, libs


def test_blt_under_graph_capture_replays():
    """A key first seen inside a hipGraph capture takes the heuristic pick (no timing under
    capture); replays compute the right product."""
    g = torch.Generator(device="cuda").manual_seed(3)
    a = (torch.randn(333, 200, device="cuda", generator=g) * 0.1).to(BF)
    b = (torch.randn(200, 176, device="cuda", generator=g) * 0.1).to(BF)
    out = torch.zeros(333, 176, device="cuda", dtype=F32)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        gemm(out, a, b)  # eager first: the stream's workspace is allocated here
    torch.cuda.current_stream().wait_stream(s)
    gr = torch.cuda.CUDAGraph()
    c = (torch.randn(333, 200, device="cuda", generator=g) * 0.1).to(BF)
    with capture_guard(), torch.cuda.graph(gr):
        gemm(out, c, b, 1.0)
    out.zero_()
    gr.replay()
    torch.cuda.synchronize()
    torch.testing.assert_close(out, _ref(c, b), rtol=2e-3, atol=1e-3)


def test_blt_long_k_wgrad_captured_on_a_fresh_stream():
    """The bench's encoder weight gradient (K = 102400) first seen inside a capture on a stream
    with no workspace of its own: the capture stream takes a spare workspace, so the solution
    the library returns (a stream-K one that needs a workspace) never runs with a null one."""
    g = torch.Generator(device="cuda").manual_seed(11)
    K, M, N = 102400, 128, 1024
    a = (torch.randn(K, M, device="cuda", generator=g) * 0.1).to(BF)
    b = (torch.randn(K, N, device="cuda", generator=g) * 0.1).to(BF)
    out = torch.zeros(M, N, device="cuda", dtype=F32)
    gr = torch.cuda.CUDAGraph()
    with capture_guard(), torch.cuda.graph(gr, stream=torch.cuda.Stream()):
        gemm(out, a.t(), b)
    gr.replay()
    torch.cuda.synchronize()
    torch.testing.assert_close(out, _ref(a.t(), b), rtol=2e-3, atol=2e-2)
