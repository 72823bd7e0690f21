// torch op registrations for the gfx950 kernels: torch.ops.tsamd.<name>(...).
// Every op launches on the current HIP stream (so it is capturable into a hipGraph via
// torch.cuda.graph) and validates shapes/dtypes on the host before launch: a kernel
// never sees operand shapes other than the ones its grid assumes.
#include <torch/library.h>
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <algorithm>
#include <optional>

#include "launchers.h"

using at::Tensor;
using OT = std::optional<Tensor>;

namespace {

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

void chk(const Tensor& t, at::ScalarType dt, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == dt, name, " has dtype ", t.scalar_type(), ", expected ", dt);
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}
template <typename T>
T* P(const Tensor& t) { return reinterpret_cast<T*>(t.data_ptr()); }
template <typename T>
T* PO(const OT& t) { return t.has_value() && t->defined() ? reinterpret_cast<T*>(t->data_ptr()) : nullptr; }
void numel_eq(const Tensor& t, int64_t n, const char* name) {
  TORCH_CHECK(t.numel() == n, name, " has ", t.numel(), " elements, expected ", n);
}
void chko(const OT& t, at::ScalarType dt, int64_t n, const char* name) {
  if (t.has_value() && t->defined()) { chk(*t, dt, name); numel_eq(*t, n, name); }
}
const auto F32 = at::kFloat;
const auto BF = at::kBFloat16;
const auto I32 = at::kInt;

// ---------------------------------------------------------------- encoder LSTM
void lstm_enc_fwd_step(const Tensor& gx, const Tensor& bias, const Tensor& Wt, const Tensor& hs, const Tensor& cs,
                       const Tensor& acts, const Tensor& out, const Tensor& lens, int64_t s, int64_t T, int64_t B,
                       int64_t H) {
  chk(gx, F32, "gx"); chk(bias, F32, "bias"); numel_eq(bias, 2 * 4 * H, "bias"); chk(Wt, BF, "Wt"); chk(hs, BF, "hs"); chk(cs, F32, "cs"); chk(acts, F32, "acts");
  chk(out, BF, "out"); chk(lens, I32, "lens");
  TORCH_CHECK(H % 32 == 0 && s >= 0 && s < T, "bad lstm args");
  numel_eq(gx, 2 * T * B * 4 * H, "gx"); numel_eq(Wt, 2 * 4 * H * H, "Wt");
  numel_eq(hs, 2 * (T + 1) * B * H, "hs"); numel_eq(cs, 2 * (T + 1) * B * H, "cs");
  numel_eq(acts, 2 * T * B * 4 * H, "acts"); numel_eq(out, B * T * 2 * H, "out"); numel_eq(lens, B, "lens");
  launch_lstm_enc_fwd_step(P<float>(gx), P<float>(bias), P<bf16>(Wt), P<bf16>(hs), P<float>(cs), P<float>(acts), P<bf16>(out),
                           P<int>(lens), s, T, B, H, stream());
}

void lstm_enc_bwd_step(const Tensor& dz, const Tensor& Wn, const Tensor& dout, const Tensor& dh_fin,
                       const Tensor& dc_carry, const Tensor& acts, const Tensor& cs, const Tensor& lens, int64_t s,
                       int64_t T, int64_t B, int64_t H) {
  chk(dz, BF, "dz"); chk(Wn, BF, "Wn"); chk(dout, F32, "dout"); chk(dh_fin, F32, "dh_fin");
  chk(dc_carry, F32, "dc_carry"); chk(acts, F32, "acts"); chk(cs, F32, "cs"); chk(lens, I32, "lens");
  TORCH_CHECK(H % 32 == 0 && s >= 0 && s < T, "bad lstm args");
  numel_eq(dz, 2 * T * B * 4 * H, "dz"); numel_eq(Wn, 2 * 4 * H * H, "Wn"); numel_eq(dout, B * T * 2 * H, "dout");
  numel_eq(dh_fin, 2 * B * H, "dh_fin"); numel_eq(dc_carry, 2 * B * H, "dc_carry");
  numel_eq(acts, 2 * T * B * 4 * H, "acts"); numel_eq(cs, 2 * (T + 1) * B * H, "cs");
  launch_lstm_enc_bwd_step(P<bf16>(dz), P<bf16>(Wn), P<float>(dout), P<float>(dh_fin), P<float>(dc_carry),
                           P<float>(acts), P<float>(cs), P<int>(lens), s, T, B, H, stream());
}

// persistent (one launch for all T steps) variants; see lstm_persistent.hip
int64_t lstm_persistent_grid_op(int64_t H, int64_t B) { return lstm_persistent_grid((int)H, (int)B); }
int64_t lstm_persistent_capacity_op(int64_t H) { return lstm_persistent_capacity((int)H); }
int64_t lstm_persistent_launches_op(int64_t H, int64_t B) { return lstm_persistent_launches((int)H, (int)B); }
int64_t lstm_persistent_xbuf_op(int64_t H, int64_t B, bool bwd) {
  return (int64_t)lstm_persistent_xbuf_elems((int)H, (int)B, bwd);
}

void lstm_fwd_persistent(const Tensor& gx, const Tensor& bias, const Tensor& Wt, const Tensor& hs, const Tensor& cs,
                         const Tensor& acts, const Tensor& out, const Tensor& lens, const Tensor& xbuf,
                         const Tensor& err, int64_t T, int64_t B, int64_t H) {
  chk(gx, F32, "gx"); chk(bias, F32, "bias"); numel_eq(bias, 2 * 4 * H, "bias"); chk(Wt, BF, "Wt"); chk(hs, BF, "hs"); chk(cs, F32, "cs"); chk(acts, F32, "acts");
  chk(out, BF, "out"); chk(lens, I32, "lens"); chk(xbuf, at::kLong, "xbuf"); chk(err, I32, "err");
  TORCH_CHECK(lstm_persistent_grid((int)H, (int)B) > 0, "persistent LSTM: unsupported H/B (H in {64,128,256,512}; "
              "a launch's grid must fit the resident capacity, one workgroup per CU)");
  TORCH_CHECK(T >= 1 && T < (1 << 30), "bad T");
  numel_eq(gx, 2 * T * B * 4 * H, "gx"); numel_eq(Wt, 2 * 4 * H * H, "Wt");
  numel_eq(hs, 2 * (T + 1) * B * H, "hs"); numel_eq(cs, 2 * (T + 1) * B * H, "cs");
  numel_eq(acts, 2 * T * B * 4 * H, "acts"); numel_eq(out, B * T * 2 * H, "out"); numel_eq(lens, B, "lens");
  TORCH_CHECK(xbuf.numel() >= (int64_t)lstm_persistent_xbuf_elems((int)H, (int)B, false), "xbuf too small");
  numel_eq(err, 1, "err");
  launch_lstm_fwd_persistent(P<float>(gx), P<float>(bias), P<bf16>(Wt), P<bf16>(hs), P<float>(cs), P<float>(acts), P<bf16>(out),
                             P<int>(lens), (unsigned long long*)xbuf.data_ptr(), (unsigned*)err.data_ptr(), T, B, H,
                             stream());
}

// the input projection of encoder layer 0 inside the recurrence: xsf = step-frame inputs
// [2][T][B][128] (bf16), Wx0 / Wx1 = W_x^T of each direction [4H][128] (row u * 4 + g)
bool lstm_persistent_fx_ok_op(int64_t H, int64_t B, int64_t E) { return lstm_persistent_fx_ok((int)H, (int)B, (int)E); }
void lstm_fwd_persistent_fx(const Tensor& xsf, const Tensor& Wx0, const Tensor& Wx1, const Tensor& bias,
                            const Tensor& Wt, const Tensor& hs, const Tensor& cs, const Tensor& acts, const Tensor& out,
                            const Tensor& lens, const Tensor& xbuf, const Tensor& err, int64_t T, int64_t B, int64_t H) {
  chk(xsf, BF, "xsf"); chk(Wx0, BF, "Wx0"); chk(Wx1, BF, "Wx1");
  chk(bias, F32, "bias"); numel_eq(bias, 2 * 4 * H, "bias"); chk(Wt, BF, "Wt"); chk(hs, BF, "hs"); chk(cs, F32, "cs");
  chk(acts, F32, "acts"); chk(out, BF, "out"); chk(lens, I32, "lens"); chk(xbuf, at::kLong, "xbuf"); chk(err, I32, "err");
  TORCH_CHECK(lstm_persistent_fx_ok((int)H, (int)B, 128), "persistent LSTM with the input projection: unsupported H/B");
  TORCH_CHECK(T >= 1 && T < (1 << 30), "bad T");
  numel_eq(xsf, 2 * T * B * 128, "xsf"); numel_eq(Wx0, 4 * H * 128, "Wx0"); numel_eq(Wx1, 4 * H * 128, "Wx1");
  numel_eq(Wt, 2 * 4 * H * H, "Wt");
  numel_eq(hs, 2 * (T + 1) * B * H, "hs"); numel_eq(cs, 2 * (T + 1) * B * H, "cs");
  numel_eq(acts, 2 * T * B * 4 * H, "acts"); numel_eq(out, B * T * 2 * H, "out"); numel_eq(lens, B, "lens");
  TORCH_CHECK(xbuf.numel() >= (int64_t)lstm_persistent_xbuf_elems((int)H, (int)B, false), "xbuf too small");
  numel_eq(err, 1, "err");
  launch_lstm_fwd_persistent(nullptr, P<float>(bias), P<bf16>(Wt), P<bf16>(hs), P<float>(cs), P<float>(acts), P<bf16>(out),
                             P<int>(lens), (unsigned long long*)xbuf.data_ptr(), (unsigned*)err.data_ptr(), T, B, H,
                             stream(), P<bf16>(xsf), P<bf16>(Wx0), P<bf16>(Wx1));
}

void lstm_bwd_persistent(const Tensor& dz, const Tensor& Wn, const Tensor& dout, const Tensor& dh_fin,
                         const Tensor& dc_carry, const Tensor& acts, const Tensor& cs, const Tensor& lens,
                         const Tensor& xbuf, const Tensor& err, const OT& dbias, int64_t T, int64_t B, int64_t H,
                         bool dout_batch_frame) {
  // dout: fp32, or bf16 in the batch frame (the top layer reading the bf16 encoder-output gradient)
  const bool dout16 = dout.scalar_type() == BF;
  TORCH_CHECK(!dout16 || dout_batch_frame, "lstm_bwd_persistent: a bf16 dout is read in the batch frame only");
  chk(dz, BF, "dz"); chk(Wn, BF, "Wn"); chk(dout, dout16 ? BF : F32, "dout"); chk(dh_fin, F32, "dh_fin");
  chko(dbias, F32, 2 * 4 * H, "dbias");
  chk(dc_carry, F32, "dc_carry"); chk(acts, F32, "acts"); chk(cs, F32, "cs"); chk(lens, I32, "lens");
  chk(xbuf, at::kLong, "xbuf"); chk(err, I32, "err");
  TORCH_CHECK(lstm_persistent_grid((int)H, (int)B) > 0, "persistent LSTM: unsupported H/B");
  TORCH_CHECK(T >= 1 && T < (1 << 30), "bad T");
  numel_eq(dz, 2 * T * B * 4 * H, "dz"); numel_eq(Wn, 2 * 4 * H * H, "Wn"); numel_eq(dout, B * T * 2 * H, "dout");
  numel_eq(dh_fin, 2 * B * H, "dh_fin"); numel_eq(dc_carry, 2 * B * H, "dc_carry");
  numel_eq(acts, 2 * T * B * 4 * H, "acts"); numel_eq(cs, 2 * (T + 1) * B * H, "cs"); numel_eq(lens, B, "lens");
  TORCH_CHECK(xbuf.numel() >= (int64_t)lstm_persistent_xbuf_elems((int)H, (int)B, true), "xbuf too small");
  numel_eq(err, 1, "err");
  launch_lstm_bwd_persistent(P<bf16>(dz), P<bf16>(Wn), (const float*)dout.data_ptr(), P<float>(dh_fin),
                             P<float>(dc_carry), P<float>(acts), P<float>(cs), P<int>(lens),
                             (unsigned long long*)xbuf.data_ptr(), (unsigned*)err.data_ptr(), PO<float>(dbias), T, B, H,
                             dout_batch_frame, stream(), dout16);
}

// ---------------------------------------------------------------- attention
// rep: rows per F/E row (decode: the beam hypotheses of one article share its encoder
// features).  F/E hold B/rep rows, s/cov/e/a/ctx hold B rows, lens has B/rep entries.
void attn_score(const Tensor& F, const Tensor& s, const Tensor& v, const OT& wc, const OT& cov, const Tensor& lens,
                const Tensor& e, int64_t B, int64_t T, int64_t A, int64_t rep) {
  chk(F, BF, "F"); chk(s, F32, "s"); chk(v, F32, "v"); chk(lens, I32, "lens"); chk(e, F32, "e");
  TORCH_CHECK(A % 64 == 0 && A <= 1024 && T % 2 == 0, "attention size must be a multiple of 64 (<= 1024), T even");
  TORCH_CHECK((rep == 1 || rep == 2 || rep == 4) && B % rep == 0, "rep must be 1, 2 or 4 and divide B");
  numel_eq(F, B / rep * T * A, "F"); numel_eq(s, B * A, "s"); numel_eq(v, A, "v"); numel_eq(e, B * T, "e");
  numel_eq(lens, B / rep, "lens"); chko(wc, F32, A, "wc"); chko(cov, F32, B * T, "cov");
  launch_attn_score(P<bf16>(F), P<float>(s), P<float>(v), PO<float>(wc), PO<float>(cov), P<int>(lens), P<float>(e), B,
                    T, A, rep, stream());
}

void attn_softmax_ctx(const Tensor& e, const Tensor& E, const Tensor& lens, const OT& cov, const Tensor& a_out,
                      const OT& cov_out, const OT& covloss, const Tensor& ctx, const OT& ctx_bf, int64_t B, int64_t T,
                      int64_t A, int64_t rep) {
  chk(e, F32, "e"); chk(E, BF, "E"); chk(lens, I32, "lens"); chk(a_out, F32, "a_out"); chk(ctx, F32, "ctx");
  TORCH_CHECK((rep == 1 || rep == 2 || rep == 4) && B % rep == 0, "rep must be 1, 2 or 4 and divide B");
  TORCH_CHECK(A % 64 == 0 && T <= (rep == 1 ? 2048 : 1024), "bad attention shape");
  numel_eq(e, B * T, "e"); numel_eq(E, B / rep * T * A, "E"); numel_eq(a_out, B * T, "a_out");
  numel_eq(ctx, B * A, "ctx"); numel_eq(lens, B / rep, "lens");
  chko(cov, F32, B * T, "cov"); chko(cov_out, F32, B * T, "cov_out"); chko(covloss, F32, B, "covloss");
  chko(ctx_bf, BF, B * A, "ctx_bf");
  launch_attn_softmax_ctx(P<float>(e), P<bf16>(E), P<int>(lens), PO<float>(cov), P<float>(a_out), PO<float>(cov_out),
                          PO<float>(covloss), P<float>(ctx), PO<bf16>(ctx_bf), B, T, A, rep, stream());
}

// one workgroup per row (attention_row.hip): forward score + softmax + coverage + context in
// one launch, backward step without atomics (ds stored, not accumulated)
bool attn_row_ok(int64_t A, int64_t T) { return attn_row_supported((int)A, (int)T); }
void attn_fwd_row(const Tensor& F, const Tensor& E, const Tensor& s, const Tensor& v, const OT& wc, const OT& cov,
                  const Tensor& lens, const Tensor& a_out, const OT& cov_out, const OT& covloss, const Tensor& ctx,
                  const OT& ctx_bf, int64_t B, int64_t T, int64_t A, int64_t rep) {
  // rep: hypothesis rows per feature row (beam decode: the rep beams of an article share F/E)
  chk(F, BF, "F"); chk(E, BF, "E"); chk(s, F32, "s"); chk(v, F32, "v"); chk(lens, I32, "lens");
  chk(a_out, F32, "a_out"); chk(ctx, F32, "ctx");
  TORCH_CHECK(attn_row_supported((int)A, (int)T), "row attention needs A in {512, 1024} and T <= 2048");
  TORCH_CHECK(rep >= 1 && B % rep == 0, "attn_fwd_row: rep must divide B");
  numel_eq(F, B / rep * T * A, "F"); numel_eq(E, B / rep * T * A, "E"); numel_eq(s, B * A, "s"); numel_eq(v, A, "v");
  numel_eq(lens, B / rep, "lens"); numel_eq(a_out, B * T, "a_out"); numel_eq(ctx, B * A, "ctx");
  chko(wc, F32, A, "wc"); chko(cov, F32, B * T, "cov"); chko(cov_out, F32, B * T, "cov_out");
  chko(covloss, F32, B, "covloss"); chko(ctx_bf, BF, B * A, "ctx_bf");
  launch_attn_fwd_row(P<bf16>(F), P<bf16>(E), P<float>(s), P<float>(v), PO<float>(wc),
                      PO<float>(cov), P<int>(lens), P<float>(a_out), PO<float>(cov_out), PO<float>(covloss), P<float>(ctx),
                      PO<bf16>(ctx_bf), B, T, A, (int)rep, stream());
}
// attribution probe of the beam-decode attention forward (A = 512; tools/attn_decode_probe.py)
void attn_fwd_row_probe(const Tensor& F, const Tensor& E, const Tensor& s, const Tensor& v, const Tensor& wc,
                        const Tensor& cov, const Tensor& lens, const Tensor& a_out, const Tensor& ctx, int64_t B, int64_t T,
                        int64_t rep, int64_t probe) {
  chk(F, BF, "F"); chk(E, BF, "E"); chk(s, F32, "s"); chk(v, F32, "v"); chk(wc, F32, "wc"); chk(cov, F32, "cov");
  chk(lens, I32, "lens"); chk(a_out, F32, "a_out"); chk(ctx, F32, "ctx");
  TORCH_CHECK(rep >= 1 && B % rep == 0 && T <= 2048, "attn_fwd_row_probe: rep | B, T <= 2048");
  numel_eq(F, B / rep * T * 512, "F"); numel_eq(E, B / rep * T * 512, "E"); numel_eq(s, B * 512, "s");
  numel_eq(v, 512, "v"); numel_eq(wc, 512, "wc"); numel_eq(cov, B * T, "cov"); numel_eq(lens, B / rep, "lens");
  numel_eq(a_out, B * T, "a_out"); numel_eq(ctx, B * 512, "ctx");
  launch_attn_fwd_row_probe(P<bf16>(F), P<bf16>(E), P<float>(s), P<float>(v), P<float>(wc), P<float>(cov), P<int>(lens),
                            P<float>(a_out), P<float>(ctx), (int)B, (int)T, (int)rep, (int)probe, stream());
}
void attn_bwd_row(const Tensor& E, const Tensor& F, const Tensor& s, const Tensor& v, const OT& wc, const OT& cov,
                  const Tensor& a, const Tensor& dctx, const Tensor& ctx, const OT& Ga, const OT& dcov_next,
                  const OT& gcl, const Tensor& lens, const Tensor& de_out, const Tensor& ds, const OT& dcov_out,
                  int64_t B, int64_t T, int64_t A) {
  chk(E, BF, "E"); chk(F, BF, "F"); chk(s, F32, "s"); chk(v, F32, "v"); chk(a, F32, "a"); chk(dctx, F32, "dctx");
  chk(ctx, F32, "ctx"); chk(lens, I32, "lens"); chk(de_out, F32, "de_out"); chk(ds, F32, "ds");
  TORCH_CHECK(attn_row_supported((int)A, (int)T), "row attention needs A in {512, 1024} and T <= 2048");
  numel_eq(E, B * T * A, "E"); numel_eq(F, B * T * A, "F"); numel_eq(s, B * A, "s"); numel_eq(v, A, "v");
  numel_eq(a, B * T, "a"); numel_eq(dctx, B * A, "dctx"); numel_eq(ctx, B * A, "ctx"); numel_eq(lens, B, "lens");
  numel_eq(de_out, B * T, "de_out"); numel_eq(ds, B * A, "ds");
  chko(wc, F32, A, "wc"); chko(cov, F32, B * T, "cov"); chko(Ga, F32, B * T, "Ga");
  chko(dcov_next, F32, B * T, "dcov_next"); chko(gcl, F32, B, "gcl"); chko(dcov_out, F32, B * T, "dcov_out");
  launch_attn_bwd_row(P<bf16>(E), P<bf16>(F), P<float>(s), P<float>(v), PO<float>(wc), PO<float>(cov), P<float>(a),
                      P<float>(dctx), P<float>(ctx), PO<float>(Ga), PO<float>(dcov_next), PO<float>(gcl),
                      P<int>(lens), P<float>(de_out), P<float>(ds), PO<float>(dcov_out), B, T, A, stream());
}

// projected-context row attention (training): G = enc_out . W_in[E:] ([B, T, 128]) replaces E in
// the recurrence; the kernels output / consume g_t = sum_i a_i G_i and dx_{t+1} (attention_row.hip)
bool attn_rowp_ok(int64_t A, int64_t T, int64_t EG) { return attn_rowp_supported((int)A, (int)T, (int)EG); }
void attn_fwd_rowp(const Tensor& F, const Tensor& G, const Tensor& s, const Tensor& v, const OT& wc, const OT& cov,
                   const Tensor& lens, const Tensor& a_out, const OT& cov_out, const OT& covloss, const Tensor& gx,
                   const Tensor& gx_bf, int64_t B, int64_t T, int64_t A, const OT& dlen, int64_t step,
                   const OT& a_bf) {
  chk(F, BF, "F"); chk(G, BF, "G"); chk(s, F32, "s"); chk(v, F32, "v"); chk(lens, I32, "lens");
  chk(a_out, F32, "a_out"); chk(gx, F32, "gx"); chk(gx_bf, BF, "gx_bf"); chko(a_bf, BF, B * T, "a_bf");
  const int64_t EG = gx.numel() / std::max<int64_t>(B, 1);
  TORCH_CHECK(attn_rowp_supported((int)A, (int)T, (int)EG), "projected row attention needs A in {512, 1024}, "
              "T <= 2048 and a 128-wide projection");
  numel_eq(F, B * T * A, "F"); numel_eq(G, B * T * EG, "G"); numel_eq(s, B * A, "s"); numel_eq(v, A, "v");
  numel_eq(lens, B, "lens"); numel_eq(a_out, B * T, "a_out"); numel_eq(gx, B * EG, "gx"); numel_eq(gx_bf, B * EG, "gx_bf");
  chko(wc, F32, A, "wc"); chko(cov, F32, B * T, "cov"); chko(cov_out, F32, B * T, "cov_out");
  chko(covloss, F32, B, "covloss"); chko(dlen, I32, B, "dlen");
  launch_attn_fwd_rowp(P<bf16>(F), P<bf16>(G), P<float>(s), P<float>(v), PO<float>(wc), PO<float>(cov), P<int>(lens),
                       P<float>(a_out), PO<float>(cov_out), PO<float>(covloss), P<float>(gx), P<bf16>(gx_bf), B, T, A,
                       PO<int>(dlen), (int)step, stream(), PO<bf16>(a_bf));
}
void attn_bwd_rowp(const Tensor& G, const Tensor& F, const Tensor& s, const Tensor& v, const OT& wc, const OT& cov,
                   const Tensor& a, const OT& dx, const Tensor& gv, const OT& Ga, const OT& dcov_next, const OT& gcl,
                   const Tensor& lens, const Tensor& de_out, const Tensor& ds, const OT& dcov_out, int64_t B, int64_t T,
                   int64_t A, const OT& dlen, int64_t step) {
  chk(G, BF, "G"); chk(F, BF, "F"); chk(s, F32, "s"); chk(v, F32, "v"); chk(a, F32, "a"); chk(gv, F32, "gv");
  chk(lens, I32, "lens"); chk(de_out, F32, "de_out"); chk(ds, F32, "ds");
  const int64_t EG = gv.numel() / std::max<int64_t>(B, 1);
  TORCH_CHECK(attn_rowp_supported((int)A, (int)T, (int)EG), "projected row attention needs A in {512, 1024}, "
              "T <= 2048 and a 128-wide projection");
  numel_eq(G, B * T * EG, "G"); numel_eq(F, B * T * A, "F"); numel_eq(s, B * A, "s"); numel_eq(v, A, "v");
  numel_eq(a, B * T, "a"); numel_eq(gv, B * EG, "gv"); numel_eq(lens, B, "lens");
  numel_eq(de_out, B * T, "de_out"); numel_eq(ds, B * A, "ds");
  chko(dx, F32, B * EG, "dx"); chko(wc, F32, A, "wc"); chko(cov, F32, B * T, "cov"); chko(Ga, F32, B * T, "Ga");
  chko(dcov_next, F32, B * T, "dcov_next"); chko(gcl, F32, B, "gcl"); chko(dcov_out, F32, B * T, "dcov_out");
  chko(dlen, I32, B, "dlen");
  launch_attn_bwd_rowp(P<bf16>(G), P<bf16>(F), P<float>(s), P<float>(v), PO<float>(wc), PO<float>(cov), P<float>(a),
                       PO<float>(dx), P<float>(gv), PO<float>(Ga), PO<float>(dcov_next), PO<float>(gcl), P<int>(lens),
                       P<float>(de_out), P<float>(ds), PO<float>(dcov_out), B, T, A, PO<int>(dlen), (int)step, stream());
}

void attn_bwd_step(const Tensor& E, const Tensor& F, const Tensor& s, const Tensor& v, const OT& wc, const OT& cov,
                   const Tensor& a, const Tensor& dctx, const Tensor& ctx, const OT& Ga, const OT& dcov_next,
                   const OT& gcl, const Tensor& lens, const Tensor& de_out, const Tensor& ds, const OT& dcov_out,
                   int64_t B, int64_t T, int64_t A) {
  chk(E, BF, "E"); chk(F, BF, "F"); chk(s, F32, "s"); chk(v, F32, "v"); chk(a, F32, "a"); chk(dctx, F32, "dctx");
  chk(ctx, F32, "ctx"); chk(lens, I32, "lens"); chk(de_out, F32, "de_out"); chk(ds, F32, "ds");
  TORCH_CHECK(A % 64 == 0 && A <= 1024 && T >= 1, "bad A/T");
  numel_eq(E, B * T * A, "E"); numel_eq(F, B * T * A, "F"); numel_eq(s, B * A, "s"); numel_eq(v, A, "v");
  numel_eq(a, B * T, "a"); numel_eq(dctx, B * A, "dctx"); numel_eq(ctx, B * A, "ctx"); numel_eq(lens, B, "lens");
  numel_eq(de_out, B * T, "de_out"); numel_eq(ds, B * A, "ds");
  chko(wc, F32, A, "wc"); chko(cov, F32, B * T, "cov"); chko(Ga, F32, B * T, "Ga");
  chko(dcov_next, F32, B * T, "dcov_next"); chko(gcl, F32, B, "gcl"); chko(dcov_out, F32, B * T, "dcov_out");
  launch_attn_bwd_step(P<bf16>(E), P<bf16>(F), P<float>(s), P<float>(v), PO<float>(wc), PO<float>(cov), P<float>(a),
                       P<float>(dctx), P<float>(ctx), PO<float>(Ga), PO<float>(dcov_next), PO<float>(gcl),
                       P<int>(lens), P<float>(de_out), P<float>(ds), PO<float>(dcov_out), B, T, A, stream());
}

void attn_bwd_feat(const Tensor& F, const Tensor& S_all, const Tensor& v, const OT& wc, const OT& cov_all,
                   const Tensor& de_all, const Tensor& lens, const Tensor& dF, const Tensor& dv, const OT& dwc,
                   int64_t D, int64_t B, int64_t T, int64_t A, const OT& dlen) {
  chk(F, BF, "F"); chk(S_all, F32, "S_all"); chk(v, F32, "v"); chk(de_all, F32, "de_all"); chk(lens, I32, "lens");
  chk(dF, BF, "dF"); chk(dv, F32, "dv");
  TORCH_CHECK(A % 64 == 0, "bad A");
  numel_eq(F, B * T * A, "F"); numel_eq(S_all, D * B * A, "S_all"); numel_eq(de_all, D * B * T, "de_all");
  // dv / dwc: [nslot][A] partial rows (nslot a power of two; the caller sums them).  With nslot >=
  // the number of workgroups every slot has one writer (deterministic mode)
  const int64_t nslot = dv.numel() / A;
  TORCH_CHECK(nslot >= 1 && nslot <= (1 << 20) && (nslot & (nslot - 1)) == 0 && dv.numel() == nslot * A,
              "dv: [nslot, A] with nslot a power of two");
  numel_eq(dF, B * T * A, "dF");
  chko(wc, F32, A, "wc"); chko(cov_all, F32, D * B * T, "cov_all"); chko(dwc, F32, nslot * A, "dwc");
  chko(dlen, I32, B, "dlen");
  launch_attn_bwd_feat(P<bf16>(F), P<float>(S_all), P<float>(v), PO<float>(wc), PO<float>(cov_all), P<float>(de_all),
                       P<int>(lens), P<bf16>(dF), P<float>(dv), PO<float>(dwc), D, B, T, A, (int)nslot, stream(),
                       PO<int>(dlen));
}

int64_t attn_chunks(int64_t T) { return attn_nchunk(T); }

void emb_grad_sorted(const Tensor& gemb, const Tensor& sid, const Tensor& perm, const Tensor& src0, const Tensor& src1) {
  chk(gemb, F32, "gemb"); chk(src0, F32, "src0"); chk(src1, F32, "src1");
  TORCH_CHECK(gemb.dim() == 2 && gemb.size(1) <= 512, "gemb must be [V][E], E <= 512");
  TORCH_CHECK(sid.scalar_type() == at::kInt && perm.scalar_type() == at::kInt && sid.is_contiguous() &&
              perm.is_contiguous() && sid.numel() == perm.numel(), "sid / perm int32, contiguous, one length");
  const int64_t E = gemb.size(1), V = gemb.size(0);
  TORCH_CHECK(src0.numel() % E == 0 && src1.numel() % E == 0, "src rows");
  const int64_t n0 = src0.numel() / E, n1 = src1.numel() / E;
  TORCH_CHECK(sid.numel() == n0 + n1, "sid must cover src0 and src1 rows");
  launch_emb_grad_sorted(P<float>(gemb), P<int>(sid), P<int>(perm), P<float>(src0), (int)n0, P<float>(src1),
                         (int)n1, (int)E, (int)V, stream());
}

// deterministic variant (no atomics): pf / pl are [chunks][E] fp32 scratch, chunks = ceil(rows / 64)
int64_t emb_grad_det_chunks_op(int64_t n) { return emb_grad_det_chunks((int)n); }
void emb_grad_det(const Tensor& gemb, const Tensor& sid, const Tensor& perm, const Tensor& src0, const Tensor& src1,
                  const Tensor& pf, const Tensor& pl) {
  chk(gemb, F32, "gemb"); chk(src0, F32, "src0"); chk(src1, F32, "src1"); chk(pf, F32, "pf"); chk(pl, F32, "pl");
  TORCH_CHECK(gemb.dim() == 2 && gemb.size(1) <= 512, "gemb must be [V][E], E <= 512");
  TORCH_CHECK(sid.scalar_type() == at::kInt && perm.scalar_type() == at::kInt && sid.is_contiguous() &&
              perm.is_contiguous() && sid.numel() == perm.numel(), "sid / perm int32, contiguous, one length");
  const int64_t E = gemb.size(1), V = gemb.size(0);
  TORCH_CHECK(src0.numel() % E == 0 && src1.numel() % E == 0, "src rows");
  const int64_t n0 = src0.numel() / E, n1 = src1.numel() / E;
  TORCH_CHECK(sid.numel() == n0 + n1, "sid must cover src0 and src1 rows");
  const int64_t nc = emb_grad_det_chunks((int)(n0 + n1));
  numel_eq(pf, nc * E, "pf"); numel_eq(pl, nc * E, "pl");
  launch_emb_grad_det(P<float>(gemb), P<int>(sid), P<int>(perm), P<float>(src0), (int)n0, P<float>(src1), (int)n1,
                      (int)E, (int)V, P<float>(pf), P<float>(pl), stream());
}

// ---------------------------------------------------------------- frames (frames.hip)
// out[2][T][B][W] from src rows: (ids? ids[b,tt] : b*T+tt), tt = t | rev[b,t]; columns d*doff..
void step_frame_hop(const Tensor& in, const Tensor& rev, const Tensor& out, int64_t B, int64_t T, int64_t H) {
  chk(in, F32, "in"); chk(out, F32, "out");
  TORCH_CHECK(H % 4 == 0 && B > 0 && T > 0, "step_frame_hop: H % 4 == 0");
  TORCH_CHECK(rev.scalar_type() == at::kLong && rev.is_contiguous() && rev.numel() == B * T, "rev [B,T] int64");
  numel_eq(in, 2 * T * B * 2 * H, "in"); numel_eq(out, 2 * T * B * H, "out");
  launch_step_frame_hop(P<float>(in), rev.data_ptr<int64_t>(), P<float>(out), (int)B, (int)T, (int)H, stream());
}

void to_step_frame(const Tensor& src, const OT& ids, const Tensor& rev, const Tensor& out, int64_t B, int64_t T,
                   int64_t W, int64_t doff) {
  TORCH_CHECK(src.is_cuda() && src.is_contiguous() && out.is_contiguous() && src.scalar_type() == out.scalar_type(),
              "src/out: contiguous GPU tensors of one dtype");
  TORCH_CHECK(src.scalar_type() == BF || src.scalar_type() == F32, "bf16 or fp32");
  TORCH_CHECK(rev.scalar_type() == at::kLong && rev.is_contiguous() && rev.numel() == B * T, "rev [B,T] int64");
  const int es = (int)src.element_size();
  TORCH_CHECK((W * es) % 16 == 0 && (doff * es) % 16 == 0, "rows must be 16-byte multiples");
  const int64_t S = src.size(-1);
  TORCH_CHECK(doff + W <= S && (S * es) % 16 == 0, "bad row width");
  if (ids.has_value()) {
    TORCH_CHECK(ids->scalar_type() == at::kLong && ids->is_contiguous() && ids->numel() == B * T, "ids [B,T] int64");
  } else {
    TORCH_CHECK(src.numel() == B * T * S, "src must be [B,T,S] without ids");
  }
  numel_eq(out, 2 * T * B * W, "out");
  launch_to_step_frame(src.data_ptr(), es, PO<int64_t>(ids), P<int64_t>(rev), out.data_ptr(), (int)B, (int)T, (int)W,
                       (int)S, (int)doff, src.numel() / S, stream());
}
void from_step_frame(const Tensor& in, const Tensor& rev, const Tensor& out, int64_t B, int64_t T, int64_t W) {
  chk(in, F32, "in"); chk(out, F32, "out");
  TORCH_CHECK(rev.scalar_type() == at::kLong && rev.is_contiguous() && rev.numel() == B * T, "rev [B,T] int64");
  TORCH_CHECK(W % 4 == 0, "W % 4");
  numel_eq(in, 2 * T * B * W, "in"); numel_eq(out, B * T * W, "out");
  launch_from_step_frame(P<float>(in), P<int64_t>(rev), P<float>(out), (int)B, (int)T, (int)W, stream());
}
void transpose_bta(const Tensor& in, const Tensor& out, int64_t B, int64_t T, int64_t A) {
  chk(in, BF, "in"); chk(out, BF, "out");
  TORCH_CHECK(A % 64 == 0, "A % 64");
  numel_eq(in, B * T * A, "in"); numel_eq(out, B * T * A, "out");
  launch_transpose_bta(P<bf16>(in), P<bf16>(out), (int)B, (int)T, (int)A, stream());
}
// fp32 [P][Q][R] -> [Q][P][R] fp32 (out) and bf16 (outb), either nullable, one pass
void tr01(const Tensor& in, const OT& out, const OT& outb, int64_t np_, int64_t nq, int64_t nr, bool acc) {
  chk(in, F32, "in");
  TORCH_CHECK(nr % 4 == 0 && np_ >= 1 && nq >= 1, "tr01: R % 4 == 0");
  TORCH_CHECK(!acc || (out.has_value() && !outb.has_value()), "tr01: acc adds into out (no bf16 twin)");
  numel_eq(in, np_ * nq * nr, "in");
  chko(out, F32, np_ * nq * nr, "out"); chko(outb, BF, np_ * nq * nr, "outb");
  // 16-byte fp32 vector accesses, 8-byte bf16 stores: a contiguous view at an offset (a per-step
  // slice) must still be aligned
  TORCH_CHECK((uintptr_t)in.data_ptr() % 16 == 0, "tr01: in must be 16-byte aligned");
  TORCH_CHECK(!PO<float>(out) || (uintptr_t)PO<float>(out) % 16 == 0, "tr01: out must be 16-byte aligned");
  TORCH_CHECK(!PO<bf16>(outb) || (uintptr_t)PO<bf16>(outb) % 8 == 0, "tr01: outb must be 8-byte aligned");
  launch_tr01(P<float>(in), PO<float>(out), PO<bf16>(outb), (int)np_, (int)nq, (int)nr, acc, stream());
}
void cast_colsum(const Tensor& x, const Tensor& xb, const Tensor& colsum, int64_t N, int64_t C) {
  chk(x, F32, "x"); chk(xb, BF, "xb"); chk(colsum, F32, "colsum");
  TORCH_CHECK(C % 4 == 0 && C / 4 <= 256 && 256 % (C / 4) == 0, "cast_colsum: C % 4 == 0 and C / 4 divides 256");
  numel_eq(x, N * C, "x"); numel_eq(xb, N * C, "xb"); numel_eq(colsum, C, "colsum");
  auto part = at::empty({(int64_t)cast_colsum_blocks((int)N, (int)C), C}, x.options());
  launch_cast_colsum(P<float>(x), P<bf16>(xb), P<float>(part), P<float>(colsum), (int)N, (int)C, stream());
}
// out[c] (= or += with acc) = sum_n x[n][c] in an order fixed by (N, C): x fp32 or bf16 [N][C]
void colsum(const Tensor& x, const Tensor& out, int64_t N, int64_t C, bool acc) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && (x.scalar_type() == F32 || x.scalar_type() == BF),
              "colsum: x must be a contiguous CUDA fp32 / bf16 tensor");
  chk(out, F32, "out");
  numel_eq(x, N * C, "x"); numel_eq(out, C, "out");
  auto part = at::empty({(int64_t)colsum_det_chunks((int)N, (int)C), C}, out.options());
  launch_colsum_det(x.data_ptr(), x.scalar_type() == BF, P<float>(part), P<float>(out), (int)N, (int)C, acc, stream());
}

// ---------------------------------------------------------------- reduce_states
// cs / hs: the top encoder layer's step-frame states [2][T+1][B][H]; the kernels read rows T.
void rs_fwd(const Tensor& cs, const Tensor& hs, int64_t T, const Tensor& RCt, const Tensor& RHt, const Tensor& bc,
            const Tensor& bh, const Tensor& pre_c, const Tensor& pre_h, const Tensor& c0, const Tensor& c0b,
            const Tensor& h0b, const OT& cat_c, const OT& cat_h, int64_t B, int64_t H) {
  chk(cs, F32, "cs"); chk(hs, BF, "hs"); chk(RCt, BF, "RCt"); chk(RHt, BF, "RHt"); chk(bc, F32, "bc"); chk(bh, F32, "bh");
  chk(pre_c, F32, "pre_c"); chk(pre_h, F32, "pre_h"); chk(c0, F32, "c0"); chk(c0b, BF, "c0b"); chk(h0b, BF, "h0b");
  TORCH_CHECK(H % 32 == 0 && H <= 512, "reduce_states: H % 32 == 0, H <= 512");
  numel_eq(cs, 2 * (T + 1) * B * H, "cs"); numel_eq(hs, 2 * (T + 1) * B * H, "hs");
  numel_eq(RCt, 2 * H * H, "RCt"); numel_eq(RHt, 2 * H * H, "RHt"); numel_eq(bc, H, "bc"); numel_eq(bh, H, "bh");
  numel_eq(pre_c, B * H, "pre_c"); numel_eq(pre_h, B * H, "pre_h"); numel_eq(c0, B * H, "c0");
  numel_eq(c0b, B * H, "c0b"); numel_eq(h0b, B * H, "h0b");
  chko(cat_c, BF, 2 * B * H, "cat_c"); chko(cat_h, BF, 2 * B * H, "cat_h");
  const size_t off = (size_t)T * B * H, ds = (size_t)(T + 1) * B * H;
  launch_rs_fwd(P<float>(cs) + off, P<bf16>(hs) + off, ds, P<bf16>(RCt), P<bf16>(RHt), P<float>(bc), P<float>(bh),
                P<float>(pre_c), P<float>(pre_h), P<float>(c0), P<bf16>(c0b), P<bf16>(h0b), PO<bf16>(cat_c),
                PO<bf16>(cat_h), (int)B, (int)H, stream());
}

// dold_c / dold_h: [2][B][H] (fw, bw) seeds of the encoder BPTT
void rs_bwd(const Tensor& gc, const Tensor& gh, const Tensor& pre_c, const Tensor& pre_h, const Tensor& RC,
            const Tensor& RH, const Tensor& dpc, const Tensor& dph, const OT& gbc, const OT& gbh,
            const Tensor& dold_c, const Tensor& dold_h, int64_t B, int64_t H) {
  // gbc / gbh: bias gradients accumulated with atomics, or None (the caller sums: deterministic mode)
  chk(gc, F32, "gc"); chk(gh, F32, "gh"); chk(pre_c, F32, "pre_c"); chk(pre_h, F32, "pre_h"); chk(RC, BF, "RC");
  chk(RH, BF, "RH"); chk(dpc, BF, "dpc"); chk(dph, BF, "dph"); chko(gbc, F32, H, "gbc"); chko(gbh, F32, H, "gbh");
  chk(dold_c, F32, "dold_c"); chk(dold_h, F32, "dold_h");
  TORCH_CHECK(H % 32 == 0 && H <= 512, "reduce_states: H % 32 == 0, H <= 512");
  for (const Tensor* t : {&gc, &gh, &pre_c, &pre_h, &dpc, &dph}) numel_eq(*t, B * H, "[B][H] operand");
  numel_eq(RC, 2 * H * H, "RC"); numel_eq(RH, 2 * H * H, "RH");
  numel_eq(dold_c, 2 * B * H, "dold_c"); numel_eq(dold_h, 2 * B * H, "dold_h");
  launch_rs_bwd(P<float>(gc), P<float>(gh), P<float>(pre_c), P<float>(pre_h), P<bf16>(RC), P<bf16>(RH), P<bf16>(dpc),
                P<bf16>(dph), PO<float>(gbc), PO<float>(gbh), P<float>(dold_c), P<float>(dold_h), (size_t)B * H, (int)B,
                (int)H, stream());
}

// ---------------------------------------------------------------- embedding gradient
void emb_grad(const Tensor& gemb, const Tensor& ids0, const Tensor& src0, const Tensor& ids1, const Tensor& src1) {
  chk(gemb, F32, "gemb"); chk(src0, F32, "src0"); chk(src1, F32, "src1");
  TORCH_CHECK(ids0.scalar_type() == at::kLong && ids1.scalar_type() == at::kLong && ids0.is_contiguous() &&
              ids1.is_contiguous(), "ids must be contiguous int64");
  TORCH_CHECK(gemb.dim() == 2, "gemb must be [V][E]");
  const int64_t E = gemb.size(1), V = gemb.size(0);
  numel_eq(src0, ids0.numel() * E, "src0"); numel_eq(src1, ids1.numel() * E, "src1");
  launch_emb_grad(P<float>(gemb), P<int64_t>(ids0), P<float>(src0), (int)ids0.numel(), P<int64_t>(ids1), P<float>(src1),
                  (int)ids1.numel(), (int)E, (int)V, stream());
}


// ---------------------------------------------------------------- decoder cell
void dec_cell_fwd(const Tensor& XG, const OT& ctxp, const Tensor& hprev, const Tensor& cprev, const Tensor& WcT,
                  const Tensor& c_out, const Tensor& cb_out, const Tensor& hb_out, const Tensor& act, int64_t B,
                  int64_t H, int64_t A, const OT& dlen, int64_t step) {
  chk(XG, F32, "XG"); chk(hprev, BF, "hprev"); chk(cprev, F32, "cprev"); chk(WcT, BF, "WcT"); chk(c_out, F32, "c_out");
  chk(cb_out, BF, "cb_out"); chk(hb_out, BF, "hb_out"); chk(act, F32, "act");
  TORCH_CHECK(H % 32 == 0 && A % 32 == 0, "dims must be multiples of 32");
  numel_eq(XG, B * 4 * H, "XG"); chko(ctxp, BF, B * A, "ctxp"); numel_eq(hprev, B * H, "hprev");
  numel_eq(cprev, B * H, "cprev"); numel_eq(WcT, 4 * H * (A + H), "WcT"); numel_eq(c_out, B * H, "c_out");
  numel_eq(cb_out, B * H, "cb_out"); numel_eq(hb_out, B * H, "hb_out"); numel_eq(act, B * 4 * H, "act");
  chko(dlen, I32, B, "dlen");
  launch_dec_cell_fwd(P<float>(XG), PO<bf16>(ctxp), P<bf16>(hprev), P<float>(cprev), P<bf16>(WcT), P<float>(c_out),
                      P<bf16>(cb_out), P<bf16>(hb_out), P<float>(act), B, H, A, PO<int>(dlen), (int)step, stream());
}

void dec_sproj(const Tensor& cb, const Tensor& hb, const Tensor& WsT, const Tensor& bs, const Tensor& s_out, int64_t B,
               int64_t H, int64_t A, const OT& dlen, int64_t step) {
  chk(cb, BF, "cb"); chk(hb, BF, "hb"); chk(WsT, BF, "WsT"); chk(bs, F32, "bs"); chk(s_out, F32, "s_out");
  TORCH_CHECK(H % 32 == 0 && A % 16 == 0, "bad dims");
  numel_eq(cb, B * H, "cb"); numel_eq(hb, B * H, "hb"); numel_eq(WsT, A * 2 * H, "WsT"); numel_eq(bs, A, "bs");
  numel_eq(s_out, B * A, "s_out"); chko(dlen, I32, B, "dlen");
  launch_dec_sproj(P<bf16>(cb), P<bf16>(hb), P<bf16>(WsT), P<float>(bs), P<float>(s_out), B, H, A, PO<int>(dlen),
                   (int)step, stream());
}

void dec_bwd_cell(const Tensor& ds, const Tensor& Ws, const OT& dC_dir, const OT& dH_dir, const Tensor& dh_rec,
                  const Tensor& dc_carry, const Tensor& act, const Tensor& c_now, const Tensor& c_prev,
                  const Tensor& dz, int64_t B, int64_t H, int64_t A, const OT& dlen, int64_t step) {
  chk(ds, F32, "ds"); chk(Ws, BF, "Ws"); chk(dh_rec, F32, "dh_rec"); chk(dc_carry, F32, "dc_carry");
  chk(act, F32, "act"); chk(c_now, F32, "c_now"); chk(c_prev, F32, "c_prev"); chk(dz, BF, "dz");
  TORCH_CHECK(H % 16 == 0 && A % 32 == 0, "bad dims");
  numel_eq(ds, B * A, "ds"); numel_eq(Ws, 2 * H * A, "Ws"); chko(dC_dir, F32, B * H, "dC_dir");
  chko(dH_dir, F32, B * H, "dH_dir"); numel_eq(dh_rec, B * H, "dh_rec"); numel_eq(dc_carry, B * H, "dc_carry");
  numel_eq(act, B * 4 * H, "act"); numel_eq(c_now, B * H, "c_now"); numel_eq(c_prev, B * H, "c_prev");
  numel_eq(dz, B * 4 * H, "dz"); chko(dlen, I32, B, "dlen");
  launch_dec_bwd_cell(P<float>(ds), P<bf16>(Ws), PO<float>(dC_dir), PO<float>(dH_dir), P<float>(dh_rec),
                      P<float>(dc_carry), P<float>(act), P<float>(c_now), P<float>(c_prev), P<bf16>(dz), B, H, A,
                      PO<int>(dlen), (int)step, stream());
}

void dec_bwd_dz(const Tensor& dz, const Tensor& Wbig, const OT& dX_dir, const OT& dCTX_dir_prev, const Tensor& dx_out,
                const OT& dctx_prev_out, const Tensor& dh_rec, int64_t B, int64_t E, int64_t H, int64_t A,
                const OT& dlen, int64_t step) {
  chk(dz, BF, "dz"); chk(Wbig, BF, "Wbig"); chk(dx_out, F32, "dx_out"); chk(dh_rec, F32, "dh_rec");
  TORCH_CHECK(E % 16 == 0 && H % 32 == 0 && A % 16 == 0, "bad dims");
  numel_eq(dz, B * 4 * H, "dz"); numel_eq(Wbig, (E + H + A) * 4 * H, "Wbig");
  chko(dX_dir, F32, B * E, "dX_dir"); chko(dCTX_dir_prev, F32, B * A, "dCTX_dir_prev");
  numel_eq(dx_out, B * E, "dx_out"); chko(dctx_prev_out, F32, B * A, "dctx_prev_out");
  numel_eq(dh_rec, B * H, "dh_rec"); chko(dlen, I32, B, "dlen");
  launch_dec_bwd_dz(P<bf16>(dz), P<bf16>(Wbig), PO<float>(dX_dir), PO<float>(dCTX_dir_prev), P<float>(dx_out),
                    PO<float>(dctx_prev_out), P<float>(dh_rec), B, E, H, A, PO<int>(dlen), (int)step, stream());
}

// ---------------------------------------------------------------- loss / optimizer
// logits fp32 + bias (two-pass kernel), or bf16 with the bias already added (bias = None,
// one-pass kernel; dlogits may be the logits tensor itself: dz is written in place)
void ptr_loss(const Tensor& logits, const OT& bias, const Tensor& target, const Tensor& rowg, const OT& pgen,
              const OT& attn, const Tensor& ext, const Tensor& lens, const Tensor& loss_row, const OT& dlogits,
              const OT& dpre, const OT& dA, int64_t N, int64_t B, int64_t T, int64_t V) {
  const bool lbf = logits.scalar_type() == at::kBFloat16;
  chk(logits, lbf ? BF : F32, "logits"); chk(target, I32, "target"); chk(rowg, F32, "rowg"); chk(ext, I32, "ext");
  chk(lens, I32, "lens"); chk(loss_row, F32, "loss_row");
  TORCH_CHECK(lbf != bias.has_value(), "bf16 logits carry their bias (pass None); fp32 logits need the bias");
  chko(bias, F32, V, "bias");
  numel_eq(logits, N * V, "logits"); numel_eq(target, N, "target"); numel_eq(rowg, N, "rowg");
  numel_eq(ext, B * T, "ext"); numel_eq(lens, B, "lens"); numel_eq(loss_row, N, "loss_row");
  TORCH_CHECK(N % B == 0, "N must be D*B");
  chko(pgen, F32, N, "pgen"); chko(attn, F32, N * T, "attn"); chko(dlogits, BF, N * V, "dlogits");
  chko(dpre, F32, N, "dpre"); chko(dA, F32, N * T, "dA");
  TORCH_CHECK(!PO<float>(pgen) || (PO<float>(attn) && (!PO<bf16>(dlogits) || (PO<float>(dpre) && PO<float>(dA)))),
              "pointer mode needs attn, and dpre/dA when computing grads");
  if (lbf) {
    TORCH_CHECK(V <= ptr_loss_bf16_max_vocab(), "bf16 ptr_loss: V <= 65536");
    launch_ptr_loss_bf16(P<bf16>(logits), P<int>(target), P<float>(rowg), PO<float>(pgen), PO<float>(attn),
                         P<int>(ext), P<int>(lens), P<float>(loss_row), PO<bf16>(dlogits), PO<float>(dpre),
                         PO<float>(dA), N, B, T, V, stream());
    return;
  }
  launch_ptr_loss(P<float>(logits), P<float>(*bias), P<int>(target), P<float>(rowg), PO<float>(pgen), PO<float>(attn),
                  P<int>(ext), P<int>(lens), P<float>(loss_row), PO<bf16>(dlogits), PO<float>(dpre), PO<float>(dA), N,
                  B, T, V, stream());
}

// weight gradient out[M][N] += a[K][M]^T . b[K][N] (wgrad.hip): 2-D row-major views with unit
// column stride (row strides free), out fp32 and already zero (split-K atomics)
// out[Ma][Nb] (= or +=) a[K][Ma]^T . b[K][Nb] by wgrad_tt (256 x 256 / 128 tiles, split-K into the
// fp32 workspace ws, summed in split order: deterministic).  The operand roles are swapped when
// only Nb is a multiple of 256 (the slab is then summed transposed).  Returns false (nothing
// launched) for shapes it does not take.
// workspace floats for out [M][N] (acc = false; 0: shape not supported; 1: one split, the kernel
// stores straight into out)
int64_t wgrad_tt_ws(int64_t M, int64_t N, int64_t K) {
  if (wgrad_tt_ok((int)M, (int)N, (int)K))
    return wgrad_tt_direct((int)M, (int)N, (int)K, false, false) ? 1
                                                                 : (int64_t)wgrad_tt_splits((int)M, (int)N, (int)K) * M * N;
  if (wgrad_tt_ok((int)N, (int)M, (int)K)) return (int64_t)wgrad_tt_splits((int)N, (int)M, (int)K) * M * N;
  return 0;
}
bool wgrad_tt(const Tensor& a, const Tensor& b, const Tensor& out, const Tensor& ws, bool acc) {
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && out.dim() == 2, "wgrad_tt: 2-D views");
  TORCH_CHECK(a.is_cuda() && b.is_cuda() && out.is_cuda() && ws.is_cuda(), "wgrad_tt: GPU tensors");
  TORCH_CHECK(a.scalar_type() == BF && b.scalar_type() == BF && out.scalar_type() == F32 && ws.scalar_type() == F32,
              "wgrad_tt: bf16, bf16 -> fp32");
  TORCH_CHECK(a.stride(1) == 1 && b.stride(1) == 1 && out.stride(1) == 1 && ws.is_contiguous(), "wgrad_tt: unit column stride");
  const int64_t K = a.size(0), M = a.size(1), N = b.size(1), nv = out.size(1);
  // out may be narrower than b (nv < N: b's columns past nv are K-padding of a 128-aligned
  // operand, e.g. the vocab dlogits rows; those output columns are dropped)
  TORCH_CHECK(b.size(0) == K && out.size(0) == M && nv <= N, "wgrad_tt: shapes");
  if (!(a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0 && (uintptr_t)a.data_ptr() % 16 == 0 &&
        (uintptr_t)b.data_ptr() % 16 == 0))
    return false;  // 16-byte aligned operand rows only (the caller takes its other path); out: any
  const bool plain = wgrad_tt_ok((int)M, (int)N, (int)K), swapped = !plain && wgrad_tt_ok((int)N, (int)M, (int)K);
  if (!plain && !(swapped && nv == N)) return false;
  if (nv != N && (nv % 4 != 0)) return false;
  const bool direct = plain && wgrad_tt_direct((int)M, (int)N, (int)K, false, acc);
  const int64_t need = direct ? 0 : (int64_t)wgrad_tt_splits((int)(plain ? M : N), (int)(plain ? N : M), (int)K) * M * N;
  if (ws.numel() < need) {
    TORCH_CHECK(acc, "wgrad_tt: workspace too small");
    return false;  // acc on a one-split shape needs the slab wgrad_tt_ws did not count
  }
  if (plain)
    launch_wgrad_tt(P<bf16>(a), (int)a.stride(0), P<bf16>(b), (int)b.stride(0), P<float>(ws), P<float>(out),
                    (int)out.stride(0), (int)M, (int)N, (int)K, false, acc, (int)nv, stream());
  else  // GEMM over (b, a): slab [S][N][M], summed into out [M][N] transposed
    launch_wgrad_tt(P<bf16>(b), (int)b.stride(0), P<bf16>(a), (int)a.stride(0), P<float>(ws), P<float>(out),
                    (int)out.stride(0), (int)N, (int)M, (int)K, true, acc, (int)M, stream());
  return true;
}
// batched attention-context GEMMs (ctx_bmm.hip): att / dctx step-major [D][B][T] / [D][B][A] bf16,
// enc [B][T][A] bf16; outputs fp32 (ctx_fwd also the bf16 twin)
bool ctx_bmm_ok_op(int64_t B, int64_t T, int64_t D, int64_t A) { return ctx_bmm_ok((int)B, (int)T, (int)D, (int)A); }
static void ctx_chk(const Tensor& t, at::ScalarType dt, int64_t n, const char* name) {
  chk(t, dt, name);
  numel_eq(t, n, name);
  TORCH_CHECK((uintptr_t)t.data_ptr() % 16 == 0, name, ": 16-byte aligned base");
}
void ctx_fwd(const Tensor& att, const Tensor& enc, const Tensor& ctx, const Tensor& ctxb, int64_t B, int64_t T, int64_t D,
             int64_t A) {
  TORCH_CHECK(ctx_bmm_ok((int)B, (int)T, (int)D, (int)A), "ctx_fwd: D <= 128, T % 8 == 0, A % 128 == 0");
  ctx_chk(att, BF, D * B * T, "att"); ctx_chk(enc, BF, B * T * A, "enc");
  ctx_chk(ctx, F32, D * B * A, "ctx"); ctx_chk(ctxb, BF, D * B * A, "ctxb");
  launch_ctx_fwd(P<bf16>(att), P<bf16>(enc), P<float>(ctx), P<bf16>(ctxb), (int)B, (int)T, (int)D, (int)A, stream());
}
void ctx_da(const Tensor& dctx, const Tensor& enc, const Tensor& da, int64_t B, int64_t T, int64_t D, int64_t A, bool acc) {
  TORCH_CHECK(ctx_bmm_ok((int)B, (int)T, (int)D, (int)A), "ctx_da: D <= 128, T % 8 == 0, A % 128 == 0");
  ctx_chk(dctx, BF, D * B * A, "dctx"); ctx_chk(enc, BF, B * T * A, "enc"); ctx_chk(da, F32, D * B * T, "da");
  launch_ctx_da(P<bf16>(dctx), P<bf16>(enc), P<float>(da), (int)B, (int)T, (int)D, (int)A, acc, stream());
}
// dE = a^T . dctx into an fp32 or a bf16 de
void ctx_de(const Tensor& att, const Tensor& dctx, const Tensor& de, int64_t B, int64_t T, int64_t D, int64_t A) {
  TORCH_CHECK(ctx_bmm_ok((int)B, (int)T, (int)D, (int)A), "ctx_de: D <= 128, T % 8 == 0, A % 128 == 0");
  const bool b16 = de.scalar_type() == BF;
  ctx_chk(att, BF, D * B * T, "att"); ctx_chk(dctx, BF, D * B * A, "dctx"); ctx_chk(de, b16 ? BF : F32, B * T * A, "de");
  launch_ctx_de(P<bf16>(att), P<bf16>(dctx), b16 ? nullptr : P<float>(de), b16 ? P<bf16>(de) : nullptr, (int)B, (int)T,
                (int)D, (int)A, stream());
}
void wgrad_tn(const Tensor& a, const Tensor& b, const Tensor& out) {
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && out.dim() == 2, "wgrad_tn: 2-D views");
  TORCH_CHECK(a.is_cuda() && b.is_cuda() && out.is_cuda(), "wgrad_tn: GPU tensors");
  TORCH_CHECK(a.scalar_type() == BF && b.scalar_type() == BF && out.scalar_type() == F32, "wgrad_tn: bf16, bf16 -> fp32");
  TORCH_CHECK(a.stride(1) == 1 && b.stride(1) == 1 && out.stride(1) == 1, "wgrad_tn: unit column stride");
  const int64_t K = a.size(0), M = a.size(1), N = b.size(1);
  TORCH_CHECK(b.size(0) == K && out.size(0) == M && out.size(1) == N, "wgrad_tn: shapes");
  TORCH_CHECK(M % 128 == 0 && N % 8 == 0 && K >= 1, "wgrad_tn: M a multiple of 128, N of 8");
  TORCH_CHECK(a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0 && (uintptr_t)a.data_ptr() % 16 == 0 &&
              (uintptr_t)b.data_ptr() % 16 == 0, "wgrad_tn: 16-byte aligned rows");
  launch_wgrad_tn(P<bf16>(a), (int)a.stride(0), P<bf16>(b), (int)b.stride(0), P<float>(out), (int)out.stride(0),
                  (int)M, (int)N, (int)K, stream());
}

// weight repack (pack.hip): jobs [nj][13] int64 on the device (see the kernel for the layout)
int64_t pack_max_jobs_op() { return pack_max_jobs(); }
int64_t pack_job_cols_op() { return pack_job_cols(); }
// total: the number of workgroups (sum of the jobs' block counts, pack.hip)
void pack_cast(const Tensor& jobs, int64_t total) {
  TORCH_CHECK(jobs.is_cuda() && jobs.scalar_type() == at::kLong && jobs.is_contiguous() && jobs.dim() == 2 &&
              jobs.size(1) == pack_job_cols(), "pack_cast: jobs [nj][", pack_job_cols(), "] int64 on the GPU");
  TORCH_CHECK(jobs.size(0) >= 1 && jobs.size(0) <= pack_max_jobs(), "pack_cast: 1..", pack_max_jobs(), " jobs");
  launch_pack_cast(P<long>(jobs), (int)jobs.size(0), (long)total, stream());
}

// debug build (dcheck.h / debug.hip): first failed bounds check (id, block, thread, value)
int64_t debug_enabled() { return tsamd_debug_enabled(); }
Tensor debug_status() {
  unsigned v[4];
  tsamd_debug_read(v);  // synchronous copy from the device record
  Tensor t = at::empty({4}, at::TensorOptions().dtype(at::kLong));
  int64_t* d = t.data_ptr<int64_t>();
  for (int i = 0; i < 4; ++i) d[i] = (int64_t)v[i];
  return t;
}
void debug_clear() { tsamd_debug_clear(); }

// ---------------------------------------------------------------- hand-written MFMA GEMM (gemm_mfma.hip)
// out[M, N] (+)= A[arow(m), :K] . Bt[N, K]^T (+ bias): A rows plain (ids / rev absent) or gathered
// through the encoder step frame (rev [B][T] int64, direction dir; ids [B][T] int64 optional: A is
// then the embedding table) -- every operand row-contiguous with its own leading dimension
bool gemm_bt_ok(int64_t M, int64_t N, int64_t K) { return gemm_bt_supported((int)M, (int)N, (int)K, N % 256 == 0 ? 256 : 128); }
// split-K gemm_bt: out (= or +=) A . Bt^T over S K-splits into the fp32 slab ws ([S][M][N]),
// summed in split order (deterministic).  Workspace floats, 0 when the shape does not split.
int64_t gemm_bt_splitk_ws(int64_t M, int64_t N, int64_t K) {
  if (!gemm_bt_ok(M, N, K)) return 0;
  const int S = gemm_bt_splits((int)M, (int)N, (int)K);
  return S > 1 ? (int64_t)S * M * N : 0;
}
bool gemm_bt_splitk(const Tensor& A, const Tensor& Bt, const Tensor& out, const Tensor& ws, bool acc) {
  TORCH_CHECK(A.is_cuda() && A.dim() == 2 && A.scalar_type() == BF && A.stride(1) == 1, "gemm_bt_splitk: A [rows, K] bf16");
  TORCH_CHECK(Bt.is_cuda() && Bt.dim() == 2 && Bt.scalar_type() == BF && Bt.stride(1) == 1, "gemm_bt_splitk: Bt [N, K] bf16");
  TORCH_CHECK(out.is_cuda() && out.dim() == 2 && out.stride(1) == 1 && out.scalar_type() == F32, "gemm_bt_splitk: out fp32");
  TORCH_CHECK(ws.is_cuda() && ws.is_contiguous() && ws.scalar_type() == F32, "gemm_bt_splitk: fp32 workspace");
  const int64_t M = out.size(0), N = out.size(1), K = Bt.size(1);
  TORCH_CHECK(Bt.size(0) == N && A.size(1) == K && A.size(0) >= M, "gemm_bt_splitk: shape mismatch A ", A.sizes(), " Bt ",
              Bt.sizes(), " out ", out.sizes());
  const int64_t need = gemm_bt_splitk_ws(M, N, K);
  if (need == 0 || ws.numel() < need) return false;
  if (!(A.stride(0) % 8 == 0 && Bt.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(A.data_ptr()) % 16 == 0 &&
        reinterpret_cast<uintptr_t>(Bt.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0 &&
        out.stride(0) % 4 == 0))
    return false;
  launch_gemm_bt_splitk(P<bf16>(A), A.stride(0), P<bf16>(Bt), Bt.stride(0), P<float>(ws), P<float>(out), out.stride(0),
                        (int)M, (int)N, (int)K, acc, stream());
  return true;
}
void gemm_bt(const Tensor& A, const Tensor& Bt, const Tensor& out, double beta, const OT& bias, const OT& ids,
             const OT& rev, int64_t B, int64_t T, int64_t dir, const OT& xsf) {
  TORCH_CHECK(A.is_cuda() && A.dim() == 2 && A.scalar_type() == BF && A.stride(1) == 1, "gemm_bt: A [rows, K] bf16");
  TORCH_CHECK(Bt.is_cuda() && Bt.dim() == 2 && Bt.scalar_type() == BF && Bt.stride(1) == 1, "gemm_bt: Bt [N, K] bf16");
  TORCH_CHECK(out.is_cuda() && out.dim() == 2 && out.stride(1) == 1 && (out.scalar_type() == F32 || out.scalar_type() == BF),
              "gemm_bt: out [M, N] fp32 / bf16");
  const int64_t M = out.size(0), N = out.size(1), K = Bt.size(1);
  TORCH_CHECK(Bt.size(0) == N && A.size(1) >= K, "gemm_bt: shape mismatch A ", A.sizes(), " Bt ", Bt.sizes(), " out ", out.sizes());
  TORCH_CHECK(gemm_bt_ok(M, N, K), "gemm_bt: N % 128 == 0 and K % 64 == 0 (got N ", N, " K ", K, ")");
  TORCH_CHECK(A.stride(0) % 8 == 0 && Bt.stride(0) % 8 == 0 && out.stride(0) % 8 == 0 &&
              reinterpret_cast<uintptr_t>(A.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(Bt.data_ptr()) % 16 == 0 &&
              reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0, "gemm_bt: 16-byte aligned rows");
  const bool obf = out.scalar_type() == BF;
  TORCH_CHECK(beta == 0.0 || (beta == 1.0 && !obf), "gemm_bt: beta 0, or 1 with an fp32 out");
  chko(bias, F32, N, "bias");
  const bool frame = PO<int64_t>(rev) != nullptr;
  if (frame) {
    chk(*rev, at::kLong, "rev"); numel_eq(*rev, B * T, "rev");
    TORCH_CHECK(M == B * T && (dir == 0 || dir == 1), "gemm_bt: step frame needs M = T * B and dir 0 / 1");
    if (PO<int64_t>(ids)) { chk(*ids, at::kLong, "ids"); numel_eq(*ids, B * T, "ids"); }
    else TORCH_CHECK(A.size(0) == B * T, "gemm_bt: batch-frame A needs B * T rows");
    chko(xsf, BF, M * K, "xsf");
  } else {
    TORCH_CHECK(A.size(0) >= M && !PO<int64_t>(ids) && !PO<bf16>(xsf), "gemm_bt: plain A needs M rows (no xsf)");
  }
  launch_gemm_bt(P<bf16>(A), A.stride(0), P<bf16>(Bt), Bt.stride(0), out.data_ptr(), out.stride(0), obf, beta != 0.0,
                 PO<float>(bias), (int)M, (int)N, (int)K, frame ? 1 : 0, PO<int64_t>(ids), PO<int64_t>(rev), PO<bf16>(xsf), A.size(0),
                 (int)B, (int)T, (int)dir, stream());
}

// AMODE 2 (gemm_mfma.hip): out[m] = [dz[0] row | dz[1] row] . Bt^T, the rows of each k-half read at
// step t or rev[b][t] (mode bits 0 / 1), m = t * B + b or b * T + t (mode bit 2)
void gemm_bt_merge(const Tensor& dz, const Tensor& Bt, const Tensor& out, const Tensor& rev, int64_t B, int64_t T,
                   int64_t mode) {
  TORCH_CHECK(dz.is_cuda() && dz.scalar_type() == BF && dz.is_contiguous() && dz.numel() % (2 * B * T) == 0,
              "gemm_bt_merge: dz [2][T][B][Kh] bf16, contiguous");
  const int64_t Kh = dz.numel() / (2 * B * T);
  TORCH_CHECK(Bt.is_cuda() && Bt.dim() == 2 && Bt.scalar_type() == BF && Bt.stride(1) == 1 && Bt.size(1) == 2 * Kh,
              "gemm_bt_merge: Bt [N, 2 Kh] bf16");
  chk(out, F32, "out");
  TORCH_CHECK(out.dim() == 2 && out.size(0) == B * T && out.size(1) == Bt.size(0) && out.stride(1) == 1,
              "gemm_bt_merge: out [T * B, N] fp32");
  chk(rev, at::kLong, "rev");
  numel_eq(rev, B * T, "rev");
  TORCH_CHECK(mode >= 0 && mode <= 7, "gemm_bt_merge: mode bits 0-2");
  const int64_t M = B * T, N = Bt.size(0), K = 2 * Kh;
  TORCH_CHECK(Kh % 64 == 0 && gemm_bt_ok(M, N, K), "gemm_bt_merge: Kh % 64 == 0 and N % 128 == 0");
  TORCH_CHECK(Bt.stride(0) % 8 == 0 && out.stride(0) % 4 == 0 && reinterpret_cast<uintptr_t>(dz.data_ptr()) % 16 == 0 &&
              reinterpret_cast<uintptr_t>(Bt.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0,
              "gemm_bt_merge: 16-byte aligned rows");
  launch_gemm_bt(P<bf16>(dz), Kh, P<bf16>(Bt), Bt.stride(0), out.data_ptr(), out.stride(0), false, false, nullptr,
                 (int)M, (int)N, (int)K, 2, nullptr, P<int64_t>(rev), nullptr, 0, (int)B, (int)T, (int)mode, stream());
}

// ---------------------------------------------------------------- probes (probes.hip)
int64_t cu_hold_max_lds_op() { return cu_hold_max_lds(); }
void cu_hold(const Tensor& times, int64_t grid, double ms, int64_t lds_bytes) {
  chk(times, at::kLong, "times");
  numel_eq(times, 2 * grid, "times");
  TORCH_CHECK(grid >= 1 && grid <= 4096 && ms > 0 && ms <= 2000, "cu_hold: 1..4096 workgroups for at most 2 s");
  TORCH_CHECK(lds_bytes >= 0 && lds_bytes <= cu_hold_max_lds(), "cu_hold: lds_bytes above the CU's LDS");
  launch_cu_hold((int)grid, (unsigned long long)(ms * 1e5), P<long long>(times), (int)lds_bytes, stream());
}
void tanh_eval(const Tensor& x, const Tensor& t, const Tensor& s2, int64_t mode) {
  chk(x, F32, "x"); chk(t, F32, "t"); chk(s2, F32, "s2");
  numel_eq(t, x.numel(), "t"); numel_eq(s2, x.numel(), "s2");
  TORCH_CHECK(mode == 0 || mode == 1, "tanh_eval: mode 0 (exp + rcp) or 1 (rational)");
  launch_tanh_eval(P<float>(x), P<float>(t), P<float>(s2), (int)x.numel(), (int)mode, stream());
}
void tanh_tput(const Tensor& in, const Tensor& out, int64_t iters, int64_t mode) {
  chk(in, F32, "in"); chk(out, F32, "out");
  TORCH_CHECK(in.numel() >= 1024 && out.numel() % 256 == 0 && out.numel() > 0, "tanh_tput: in >= 1024, out % 256");
  TORCH_CHECK((mode == 0 || mode == 1) && iters >= 1, "tanh_tput: mode 0 / 1");
  launch_tanh_tput(P<float>(in), P<float>(out), (int)out.numel(), (int)iters, (int)mode, stream());
}

// fused training vocab head (vocab_train.hip): logits never materialised
int64_t vocab_train_tiles_op(int64_t V, int64_t H) { return vocab_train_tiles((int)V, (int)H); }

// X: [N][ldx] bf16 (the first H columns are the activations; ldx >= H, ldx % 8 == 0)
void vocab_train_fwd(const Tensor& X, const Tensor& WT, const Tensor& bias, const Tensor& target, const Tensor& part,
                     const Tensor& zg, const Tensor& lse, const Tensor& pv, int64_t N, int64_t V, int64_t H,
                     int64_t ldx, const OT& vblk, const OT& vblk_n) {
  chk(X, BF, "X"); chk(WT, BF, "WT"); chk(bias, F32, "bias"); chk(target, I32, "target"); chk(part, F32, "part");
  chk(zg, F32, "zg"); chk(lse, F32, "lse"); chk(pv, F32, "pv");
  TORCH_CHECK(H == 128 || H == 256 || H == 512, "fused training vocab head: hidden size 128, 256 or 512");
  TORCH_CHECK(N >= 1 && V >= 1 && ldx >= H && ldx % 8 == 0, "bad N/V/ldx");
  numel_eq(X, N * ldx, "X"); numel_eq(WT, V * H, "WT"); numel_eq(bias, V, "bias"); numel_eq(target, N, "target");
  numel_eq(part, (int64_t)vocab_train_tiles((int)V, (int)H) * N * 2, "part"); numel_eq(zg, N, "zg"); numel_eq(lse, N, "lse");
  numel_eq(pv, N, "pv");
  // vblk [ceil(N / 32)]: the live 32-row blocks first, *vblk_n of them (the host builds both)
  const int64_t RB = (N + 31) / 32;
  TORCH_CHECK(vblk.has_value() == vblk_n.has_value(), "vblk and vblk_n go together");
  chko(vblk, I32, RB, "vblk"); chko(vblk_n, I32, 1, "vblk_n");
  launch_vocab_train_fwd(P<bf16>(X), (int)ldx, P<bf16>(WT), P<float>(bias), P<int>(target), P<float>(part), P<float>(zg),
                         P<float>(lse), P<float>(pv), N, V, H, PO<int>(vblk), PO<int>(vblk_n), stream());
}

void vocab_train_bwd(const Tensor& X, const Tensor& WT, const Tensor& bias, const Tensor& target, const Tensor& lse,
                     const Tensor& alpha, const Tensor& dl, const OT& dbias, int64_t N, int64_t V, int64_t H,
                     int64_t ldx, const OT& vblk, const OT& vblk_n, const OT& vlive, const OT& vstate) {
  chk(X, BF, "X"); chk(WT, BF, "WT"); chk(bias, F32, "bias"); chk(target, I32, "target"); chk(lse, F32, "lse");
  chk(alpha, F32, "alpha"); chk(dl, BF, "dl");
  TORCH_CHECK(H == 128 || H == 256 || H == 512, "fused training vocab head: hidden size 128, 256 or 512");
  TORCH_CHECK(N >= 1 && V >= 1 && ldx >= H && ldx % 8 == 0, "bad N/V/ldx");
  numel_eq(X, N * ldx, "X"); numel_eq(WT, V * H, "WT"); numel_eq(bias, V, "bias"); numel_eq(target, N, "target");
  numel_eq(lse, N, "lse"); numel_eq(alpha, N, "alpha"); chko(dbias, F32, V, "dbias");
  // dlogits rows of ldd >= V elements (numel N * ldd): the columns past V are never written (the
  // caller keeps them zero: the K / N padding of the 128-aligned gradient GEMMs)
  TORCH_CHECK(dl.numel() % N == 0, "dl: numel must be N * ldd");
  const int64_t ldd = dl.numel() / N;
  TORCH_CHECK(ldd >= V && (ldd == V || ldd % 8 == 0), "dl: row length ", ldd, " must be V or a multiple of 8");
  const int64_t RB = (N + 31) / 32;
  const bool has = vblk.has_value();
  // vblk + vblk_n alone: compacted dlogits (live block j -> rows 32 j ..); with vlive + vstate: in place
  TORCH_CHECK(vblk_n.has_value() == has && vlive.has_value() == vstate.has_value() && (has || !vlive.has_value()),
              "vblk and vblk_n go together, vlive and vstate go together (and need vblk)");
  chko(vblk, I32, RB, "vblk"); chko(vblk_n, I32, 1, "vblk_n"); chko(vlive, I32, RB, "vlive");
  chko(vstate, I32, RB, "vstate");
  launch_vocab_train_bwd(P<bf16>(X), (int)ldx, P<bf16>(WT), P<float>(bias), P<int>(target), P<float>(lse), P<float>(alpha),
                         P<bf16>(dl), (int)ldd, PO<float>(dbias), N, V, H, PO<int>(vblk), PO<int>(vblk_n), PO<int>(vlive),
                         PO<int>(vstate), stream());
}

void ptr_rowfin(const Tensor& pv, const Tensor& target, const Tensor& rowg, const OT& pgen, const OT& attn,
                const Tensor& ext, const Tensor& lens, const Tensor& loss_row, const OT& alpha, const OT& dpre,
                const OT& dA, int64_t N, int64_t B, int64_t T) {
  chk(pv, F32, "pv"); chk(target, I32, "target"); chk(rowg, F32, "rowg"); chk(ext, I32, "ext"); chk(lens, I32, "lens");
  chk(loss_row, F32, "loss_row");
  TORCH_CHECK(B >= 1 && N % B == 0, "N must be D*B");
  numel_eq(pv, N, "pv"); numel_eq(target, N, "target"); numel_eq(rowg, N, "rowg"); numel_eq(ext, B * T, "ext");
  numel_eq(lens, B, "lens"); numel_eq(loss_row, N, "loss_row");
  chko(pgen, F32, N, "pgen"); chko(attn, F32, N * T, "attn"); chko(alpha, F32, N, "alpha"); chko(dpre, F32, N, "dpre");
  chko(dA, F32, N * T, "dA");
  TORCH_CHECK(!PO<float>(pgen) || PO<float>(attn), "pointer mode needs attn");
  launch_ptr_rowfin(P<float>(pv), P<int>(target), P<float>(rowg), PO<float>(pgen), PO<float>(attn), P<int>(ext),
                    P<int>(lens), P<float>(loss_row), PO<float>(alpha), PO<float>(dpre), PO<float>(dA), N, B, T,
                    stream());
}

void clip_adagrad(const Tensor& w, const Tensor& acc, const Tensor& g, const Tensor& part, double lr, double max_norm,
                  double gscale, const Tensor& norm_out, const Tensor& flag, const OT& skip) {
  chk(w, F32, "w"); chk(acc, F32, "acc"); chk(g, F32, "g"); chk(part, F32, "part"); chk(norm_out, F32, "norm_out");
  chk(flag, I32, "flag"); chko(skip, I32, 1, "skip");
  TORCH_CHECK(w.numel() == acc.numel() && w.numel() == g.numel(), "flat buffers differ in size");
  numel_eq(part, opt_nparts(), "part");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(g.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(acc.data_ptr()) % 16 == 0,
              "flat buffers must be 16-byte aligned");
  launch_clip_adagrad(P<float>(w), P<float>(acc), P<float>(g), w.numel(), P<float>(part), (float)lr, (float)max_norm,
                      (float)gscale, P<float>(norm_out), P<int>(flag), PO<int>(skip), stream());
}
int64_t opt_parts() { return opt_nparts(); }

// ---------------------------------------------------------------- beam search
void final_topk(const Tensor& logits, const Tensor& bias, const OT& pgen, const OT& attn, const Tensor& ext,
                const Tensor& lens, const Tensor& out_ids, const Tensor& out_lp, const Tensor& part_ms,
                const Tensor& part_v, const Tensor& part_i, int64_t R, int64_t V, int64_t T, int64_t K, int64_t beam) {
  chk(logits, F32, "logits"); chk(bias, F32, "bias"); chk(ext, I32, "ext"); chk(lens, I32, "lens");
  chk(out_ids, I32, "out_ids"); chk(out_lp, F32, "out_lp"); chk(part_ms, F32, "part_ms"); chk(part_v, F32, "part_v");
  chk(part_i, I32, "part_i");
  TORCH_CHECK(K >= 1 && K <= 16 && beam >= 1 && R % beam == 0 && T <= 2048, "bad topk args");
  numel_eq(logits, R * V, "logits"); numel_eq(bias, V, "bias"); numel_eq(ext, (R / beam) * T, "ext");
  numel_eq(lens, R / beam, "lens"); numel_eq(out_ids, R * K, "out_ids"); numel_eq(out_lp, R * K, "out_lp");
  TORCH_CHECK(topk_split(V) <= 64, "vocab too large for final_topk");
  numel_eq(part_ms, R * topk_split(V) * 2, "part_ms"); numel_eq(part_v, R * topk_split(V) * K, "part_v");
  numel_eq(part_i, R * topk_split(V) * K, "part_i");
  chko(pgen, F32, R, "pgen"); chko(attn, F32, R * T, "attn");
  TORCH_CHECK(!PO<float>(pgen) || PO<float>(attn), "pointer mode needs attn");
  launch_final_topk(P<float>(logits), P<float>(bias), PO<float>(pgen), PO<float>(attn), P<int>(ext), P<int>(lens),
                    P<int>(out_ids), P<float>(out_lp), P<float>(part_ms), P<float>(part_v), P<int>(part_i), R, V, T, K,
                    beam, stream());
}
int64_t topk_parts(int64_t V) { return topk_split(V); }

// fused decode vocab head (vocab_topk.hip): MFMA logits + tile partials, select reads K tiles per row
void vocab_topk(const Tensor& X, const Tensor& WT, const Tensor& bias, const OT& pgen, const OT& attn,
                const Tensor& ext, const Tensor& lens, const Tensor& out_ids, const Tensor& out_lp,
                const Tensor& logits, const Tensor& part_ms, int64_t R, int64_t V, int64_t H, int64_t T, int64_t K,
                int64_t beam) {
  chk(X, BF, "X"); chk(WT, BF, "WT"); chk(bias, F32, "bias"); chk(ext, I32, "ext"); chk(lens, I32, "lens");
  chk(out_ids, I32, "out_ids"); chk(out_lp, F32, "out_lp"); chk(logits, F32, "logits"); chk(part_ms, F32, "part_ms");
  const int64_t nt = vocab_topk_tiles((int)V, (int)H);
  TORCH_CHECK(K >= 1 && K <= 8 && beam >= 1 && R % beam == 0 && T <= 2048, "bad vocab_topk args (K <= 8)");
  TORCH_CHECK(H % 32 == 0 && (H <= 256 || H == 512) && nt <= 4096, "vocab_topk: H % 32 == 0, H <= 256 or 512, V <= 512k");
  numel_eq(X, R * H, "X"); numel_eq(WT, V * H, "WT"); numel_eq(bias, V, "bias");
  numel_eq(ext, (R / beam) * T, "ext"); numel_eq(lens, R / beam, "lens");
  numel_eq(out_ids, R * K, "out_ids"); numel_eq(out_lp, R * K, "out_lp");
  numel_eq(logits, R * V, "logits"); numel_eq(part_ms, R * nt * 2, "part_ms");
  chko(pgen, F32, R, "pgen"); chko(attn, F32, R * T, "attn");
  TORCH_CHECK(!PO<float>(pgen) || PO<float>(attn), "pointer mode needs attn");
  launch_vocab_topk(P<bf16>(X), P<bf16>(WT), P<float>(bias), PO<float>(pgen), PO<float>(attn), P<int>(ext),
                    P<int>(lens), P<int>(out_ids), P<float>(out_lp), P<float>(logits), P<float>(part_ms), R, V, H, T,
                    K, beam, PgIn{}, stream());
}
// vocab_topk with p_gen = sigmoid([ctx, c, h, x] . w + b) computed inside the select kernel
// (written to pg_out for the beam histories)
void vocab_topk_pg(const Tensor& X, const Tensor& WT, const Tensor& bias, const Tensor& ctx, const Tensor& c,
                   const Tensor& h, const Tensor& x, const Tensor& pg_w, const Tensor& pg_b, const Tensor& pg_out,
                   const Tensor& attn, const Tensor& ext, const Tensor& lens, const Tensor& out_ids,
                   const Tensor& out_lp, const Tensor& logits, const Tensor& part_ms, int64_t R, int64_t V, int64_t H,
                   int64_t T, int64_t K, int64_t beam, int64_t A, int64_t E) {
  chk(X, BF, "X"); chk(WT, BF, "WT"); chk(bias, F32, "bias"); chk(ext, I32, "ext"); chk(lens, I32, "lens");
  chk(out_ids, I32, "out_ids"); chk(out_lp, F32, "out_lp"); chk(logits, F32, "logits"); chk(part_ms, F32, "part_ms");
  chk(ctx, F32, "ctx"); chk(c, F32, "c"); chk(h, BF, "h"); chk(x, F32, "x"); chk(pg_w, F32, "pg_w");
  chk(pg_b, F32, "pg_b"); chk(pg_out, F32, "pg_out"); chk(attn, F32, "attn");
  const int64_t nt = vocab_topk_tiles((int)V, (int)H);
  TORCH_CHECK(K >= 1 && K <= 8 && beam >= 1 && R % beam == 0 && T <= 2048, "bad vocab_topk args (K <= 8)");
  TORCH_CHECK(H % 32 == 0 && (H <= 256 || H == 512) && nt <= 4096, "vocab_topk: H % 32 == 0, H <= 256 or 512, V <= 512k");
  numel_eq(X, R * H, "X"); numel_eq(WT, V * H, "WT"); numel_eq(bias, V, "bias");
  numel_eq(ext, (R / beam) * T, "ext"); numel_eq(lens, R / beam, "lens");
  numel_eq(out_ids, R * K, "out_ids"); numel_eq(out_lp, R * K, "out_lp");
  numel_eq(logits, R * V, "logits"); numel_eq(part_ms, R * nt * 2, "part_ms"); numel_eq(attn, R * T, "attn");
  numel_eq(ctx, R * A, "ctx"); numel_eq(c, R * H, "c"); numel_eq(h, R * H, "h"); numel_eq(x, R * E, "x");
  numel_eq(pg_w, A + 2 * H + E, "pg_w"); numel_eq(pg_b, 1, "pg_b"); numel_eq(pg_out, R, "pg_out");
  const PgIn pgi{P<float>(ctx), P<float>(c), P<bf16>(h), P<float>(x), P<float>(pg_w), P<float>(pg_b),
                 P<float>(pg_out), (int)A, (int)H, (int)E};
  launch_vocab_topk(P<bf16>(X), P<bf16>(WT), P<float>(bias), nullptr, P<float>(attn), P<int>(ext), P<int>(lens),
                    P<int>(out_ids), P<float>(out_lp), P<float>(logits), P<float>(part_ms), R, V, H, T, K, beam, pgi,
                    stream());
}
int64_t vocab_topk_parts(int64_t V, int64_t H) { return vocab_topk_tiles((int)V, (int)H); }
// attribution: per-phase s_memtime stamps of the decode select kernel into buf ([R][16] int64), or off
void lstm_bwd_stamps(const OT& buf) {
  set_lstm_bwd_stamps(buf.has_value() && buf->defined() ? (unsigned long long*)buf->data_ptr() : nullptr);
}
void vocab_select_stamps(const OT& buf) {
  set_vocab_select_stamps(buf.has_value() && buf->defined() ? (unsigned long long*)buf->data_ptr() : nullptr);
}
// attribution probe of the span logits kernel (H = 256; tools/vocab_span_probe.py)
void vocab_span_probe(const Tensor& X, const Tensor& WT, const Tensor& bias, const Tensor& logits, const Tensor& part_ms,
                      int64_t R, int64_t V, int64_t probe) {
  chk(X, BF, "X"); chk(WT, BF, "WT"); chk(bias, F32, "bias"); chk(logits, F32, "logits"); chk(part_ms, F32, "part_ms");
  numel_eq(X, R * 256, "X"); numel_eq(WT, V * 256, "WT"); numel_eq(bias, V, "bias");
  // (the span-major store probe writes [NW][R][32] floats)
  TORCH_CHECK(logits.numel() >= std::max(R * V, R * 32 * 8 * (int64_t)vocab_topk_tiles((int)V, 256)), "logits too small");
  numel_eq(part_ms, R * vocab_topk_tiles((int)V, 256) * 2, "part_ms");
  launch_vocab_span_probe(P<bf16>(X), P<bf16>(WT), P<float>(bias), P<float>(logits), P<float>(part_ms), (int)R, (int)V,
                          (int)probe, stream());
}

// One beam-decode step's head: vocab_topk (p_gen inside when the pointer inputs are given) with
// the beam bookkeeping fused into the select kernel's per-article tail (replaces vocab_topk_pg +
// beam_step).  The step counter was advanced at the start of the step (dec_cell_fwd_beam).
void vocab_topk_beam(const Tensor& X, const Tensor& WT, const Tensor& bias, const OT& ctx, const OT& c, const OT& h,
                     const OT& x, const OT& pg_w, const OT& pg_b, const OT& pg_out, const OT& attn, const Tensor& ext,
                     const Tensor& lens, const Tensor& out_ids, const Tensor& out_lp, const Tensor& logits,
                     const Tensor& part_ms, const Tensor& lp_sum, const Tensor& latest, const Tensor& gidx,
                     const Tensor& tok_hist, const Tensor& par_hist, const Tensor& done, const Tensor& res_count,
                     const Tensor& res_score, const Tensor& res_len, const Tensor& res_step, const Tensor& res_par,
                     const Tensor& step, const Tensor& art_ctr, const Tensor& gran, const Tensor& err,
                     const OT& att_hist, const OT& pg_hist, int64_t R,
                     int64_t V, int64_t H, int64_t T, int64_t K, int64_t beam, int64_t A, int64_t E, int64_t stop_id,
                     int64_t min_dec, int64_t max_dec) {
  chk(X, BF, "X"); chk(WT, BF, "WT"); chk(bias, F32, "bias"); chk(ext, I32, "ext"); chk(lens, I32, "lens");
  chk(out_ids, I32, "out_ids"); chk(out_lp, F32, "out_lp"); chk(logits, F32, "logits"); chk(part_ms, F32, "part_ms");
  const int64_t nt = vocab_topk_tiles((int)V, (int)H), Na = R / beam;
  TORCH_CHECK(K >= 1 && K <= 8 && beam >= 1 && R % beam == 0 && T <= 2048 && beam * K <= 64, "bad vocab_topk_beam args");
  TORCH_CHECK(H % 32 == 0 && (H <= 256 || H == 512) && nt <= 4096, "vocab_topk: H % 32 == 0, H <= 256 or 512, V <= 512k");
  numel_eq(X, R * H, "X"); numel_eq(WT, V * H, "WT"); numel_eq(bias, V, "bias");
  numel_eq(ext, Na * T, "ext"); numel_eq(lens, Na, "lens");
  numel_eq(out_ids, R * K, "out_ids"); numel_eq(out_lp, R * K, "out_lp");
  numel_eq(logits, R * V, "logits"); numel_eq(part_ms, R * nt * 2, "part_ms"); chko(attn, F32, R * T, "attn");
  const bool ptr = pg_w.has_value() && pg_w->defined();
  PgIn pgi{};
  if (ptr) {
    chko(ctx, F32, R * A, "ctx"); chko(c, F32, R * H, "c"); chko(h, BF, R * H, "h"); chko(x, F32, R * E, "x");
    chko(pg_w, F32, A + 2 * H + E, "pg_w"); chko(pg_b, F32, 1, "pg_b"); chko(pg_out, F32, R, "pg_out");
    TORCH_CHECK(PO<float>(ctx) && PO<float>(c) && PO<bf16>(h) && PO<float>(x) && PO<float>(pg_b) && PO<float>(attn),
                "pointer mode needs ctx, c, h, x, pg_b and attn");
    pgi = PgIn{PO<float>(ctx), PO<float>(c), PO<bf16>(h), PO<float>(x), PO<float>(pg_w), PO<float>(pg_b),
               PO<float>(pg_out), (int)A, (int)H, (int)E};
  }
  chk(lp_sum, F32, "lp_sum"); chk(latest, I32, "latest"); chk(gidx, I32, "gidx"); chk(tok_hist, I32, "tok_hist");
  chk(par_hist, I32, "par_hist"); chk(done, I32, "done"); chk(res_count, I32, "res_count");
  chk(res_score, F32, "res_score"); chk(res_len, I32, "res_len"); chk(res_step, I32, "res_step");
  chk(res_par, I32, "res_par"); chk(step, I32, "step"); chk(art_ctr, I32, "art_ctr");
  numel_eq(lp_sum, R, "lp_sum"); numel_eq(latest, R, "latest"); numel_eq(gidx, R, "gidx");
  numel_eq(tok_hist, max_dec * R, "tok_hist"); numel_eq(par_hist, max_dec * R, "par_hist"); numel_eq(done, Na, "done");
  numel_eq(res_count, Na, "res_count"); numel_eq(res_score, R, "res_score"); numel_eq(res_len, R, "res_len");
  numel_eq(res_step, R, "res_step"); numel_eq(res_par, R, "res_par"); numel_eq(step, 1, "step");
  numel_eq(art_ctr, Na, "art_ctr"); chk(gran, at::kLong, "gran"); numel_eq(gran, R * K, "gran");
  chk(err, I32, "err"); numel_eq(err, 1, "err");
  TORCH_CHECK(V + T < (1 << 17), "vocab_topk_beam: extended ids must fit 17 bits");
  chko(att_hist, F32, max_dec * R * T, "att_hist"); chko(pg_hist, F32, max_dec * R, "pg_hist");
  TORCH_CHECK(!PO<float>(att_hist) || PO<float>(attn), "att_hist needs attn");
  TORCH_CHECK(!PO<float>(pg_hist) || (ptr && PO<float>(att_hist)), "pg_hist needs the pointer inputs and att_hist");
  const BeamTail bt{P<float>(lp_sum), P<int>(latest), P<int>(gidx), P<int>(tok_hist), P<int>(par_hist), P<int>(done),
                    P<int>(res_count), P<float>(res_score), P<int>(res_len), P<int>(res_step), P<int>(res_par),
                    P<int>(step), (unsigned*)P<int>(art_ctr), (unsigned long long*)gran.data_ptr(), P<int>(err),
                    PO<float>(attn), PO<float>(att_hist), PO<float>(pg_out),
                    PO<float>(pg_hist), (int)T, (int)Na, (int)beam, (int)K, (int)stop_id, (int)min_dec, (int)max_dec};
  launch_vocab_topk(P<bf16>(X), P<bf16>(WT), P<float>(bias), nullptr, ptr ? PO<float>(attn) : nullptr, P<int>(ext),
                    P<int>(lens), P<int>(out_ids), P<float>(out_lp), P<float>(logits), P<float>(part_ms), R, V, H, T, K,
                    beam, pgi, stream(), &bt);
}

// decoder cell of a beam-decode step with the parent / token gathers inside (dec_cell_fwd +
// the former beam_gather): rows read c/h/ctx of parent gidx[r] from the previous state set and
// XGtab[latest[r]]; step[0] += 1
void dec_cell_fwd_beam(const Tensor& gidx, const Tensor& latest, const Tensor& XGtab, const Tensor& ctx_src,
                       const Tensor& h_src, const Tensor& c_src, const Tensor& WcT, const Tensor& c_out,
                       const Tensor& cb_out, const Tensor& hb_out, const Tensor& step, int64_t R, int64_t H, int64_t A,
                       int64_t V, int64_t unk) {
  chk(gidx, I32, "gidx"); chk(latest, I32, "latest"); chk(XGtab, F32, "XGtab"); chk(ctx_src, BF, "ctx_src");
  chk(h_src, BF, "h_src"); chk(c_src, F32, "c_src"); chk(WcT, BF, "WcT"); chk(c_out, F32, "c_out");
  chk(cb_out, BF, "cb_out"); chk(hb_out, BF, "hb_out"); chk(step, I32, "step");
  TORCH_CHECK(H % 16 == 0 && A % 32 == 0 && H % 32 == 0 && unk >= 0 && unk < V, "bad dims");
  numel_eq(gidx, R, "gidx"); numel_eq(latest, R, "latest"); numel_eq(XGtab, V * 4 * H, "XGtab");
  numel_eq(ctx_src, R * A, "ctx_src"); numel_eq(h_src, R * H, "h_src"); numel_eq(c_src, R * H, "c_src");
  numel_eq(WcT, 4 * H * (A + H), "WcT"); numel_eq(c_out, R * H, "c_out"); numel_eq(cb_out, R * H, "cb_out");
  numel_eq(hb_out, R * H, "hb_out"); numel_eq(step, 1, "step");
  launch_dec_cell_fwd_beam(P<int>(gidx), P<int>(latest), P<float>(XGtab), P<bf16>(ctx_src), P<bf16>(h_src),
                           P<float>(c_src), P<bf16>(WcT), P<float>(c_out), P<bf16>(cb_out), P<bf16>(hb_out),
                           P<int>(step), (int)R, (int)H, (int)A, (int)V, (int)unk, stream());
}

// s = [cb, hb] . WsT^T + bs  and  x = Xtab[latest] + ctx_src[gidx] . WicT^T  in one launch
void beam_sproj_xmerge(const Tensor& cb, const Tensor& hb, const Tensor& WsT, const Tensor& bs, const Tensor& s_out,
                       const Tensor& ctx_src, const Tensor& WicT, const Tensor& Xtab, const Tensor& gidx,
                       const Tensor& latest, const Tensor& x_out, int64_t R, int64_t H, int64_t A, int64_t E,
                       int64_t V, int64_t unk) {
  chk(cb, BF, "cb"); chk(hb, BF, "hb"); chk(WsT, BF, "WsT"); chk(bs, F32, "bs"); chk(s_out, F32, "s_out");
  chk(ctx_src, BF, "ctx_src"); chk(WicT, BF, "WicT"); chk(Xtab, F32, "Xtab"); chk(gidx, I32, "gidx");
  chk(latest, I32, "latest"); chk(x_out, F32, "x_out");
  TORCH_CHECK(H % 32 == 0 && A % 32 == 0 && A % 16 == 0 && E % 16 == 0 && unk >= 0 && unk < V, "bad dims");
  numel_eq(cb, R * H, "cb"); numel_eq(hb, R * H, "hb"); numel_eq(WsT, A * 2 * H, "WsT"); numel_eq(bs, A, "bs");
  numel_eq(s_out, R * A, "s_out"); numel_eq(ctx_src, R * A, "ctx_src"); numel_eq(WicT, E * A, "WicT");
  numel_eq(Xtab, V * E, "Xtab"); numel_eq(gidx, R, "gidx"); numel_eq(latest, R, "latest"); numel_eq(x_out, R * E, "x_out");
  launch_beam_sproj_xmerge(P<bf16>(cb), P<bf16>(hb), P<bf16>(WsT), P<float>(bs), P<float>(s_out), P<bf16>(ctx_src),
                           P<bf16>(WicT), P<float>(Xtab), P<int>(gidx), P<int>(latest), P<float>(x_out), (int)R,
                           (int)H, (int)A, (int)E, (int)V, (int)unk, stream());
}

// attn_fwd_row of a beam-decode step with the coverage gather: cov = cov_src[g] + a_src[g]
// (g = gidx[row]) used for the scores and kept in cov_keep for the next step
void attn_fwd_row_beam(const Tensor& F, const Tensor& E, const Tensor& s, const Tensor& v, const OT& wc,
                       const OT& cov_src, const OT& a_src, const OT& cov_keep, const Tensor& gidx, const Tensor& lens,
                       const Tensor& a_out, const Tensor& ctx, const OT& ctx_bf, int64_t B, int64_t T, int64_t A,
                       int64_t rep) {
  chk(F, BF, "F"); chk(E, BF, "E"); chk(s, F32, "s"); chk(v, F32, "v"); chk(lens, I32, "lens"); chk(gidx, I32, "gidx");
  chk(a_out, F32, "a_out"); chk(ctx, F32, "ctx");
  TORCH_CHECK(attn_row_supported((int)A, (int)T), "row attention needs A in {512, 1024} and T <= 2048");
  TORCH_CHECK(rep >= 1 && B % rep == 0, "attn_fwd_row_beam: rep must divide B");
  numel_eq(F, B / rep * T * A, "F"); numel_eq(E, B / rep * T * A, "E"); numel_eq(s, B * A, "s"); numel_eq(v, A, "v");
  numel_eq(lens, B / rep, "lens"); numel_eq(a_out, B * T, "a_out"); numel_eq(ctx, B * A, "ctx"); numel_eq(gidx, B, "gidx");
  chko(wc, F32, A, "wc"); chko(cov_src, F32, B * T, "cov_src"); chko(a_src, F32, B * T, "a_src");
  chko(cov_keep, F32, B * T, "cov_keep"); chko(ctx_bf, BF, B * A, "ctx_bf");
  const bool cov = PO<float>(cov_src) != nullptr;
  TORCH_CHECK(cov == (PO<float>(a_src) != nullptr) && cov == (PO<float>(cov_keep) != nullptr),
              "coverage gather: cov_src, a_src and cov_keep together");
  launch_attn_fwd_row(P<bf16>(F), P<bf16>(E), P<float>(s), P<float>(v), PO<float>(wc), PO<float>(cov_src), P<int>(lens),
                      P<float>(a_out), nullptr, nullptr, P<float>(ctx), PO<bf16>(ctx_bf), B, T, A, (int)rep, stream(),
                      cov ? P<int>(gidx) : nullptr, PO<float>(a_src), PO<float>(cov_keep));
}


// Advances step[0] by one (the last block to finish) when ctr (one zeroed uint32 scratch word)
// is given; without ctr, beam_gather advanced it at the start of the decode step (t = step - 1).
// att/att_hist/pg/pg_hist (optional): this step's attention rows and p_gen copied into row
// min(step, max_dec - 1) of the histories.
void beam_step(const Tensor& top_ids, const Tensor& top_lp, const Tensor& lp_sum, const Tensor& latest,
               const Tensor& gidx, const Tensor& tok_hist, const Tensor& par_hist, const Tensor& done,
               const Tensor& res_count, const Tensor& res_score, const Tensor& res_len, const Tensor& res_step,
               const Tensor& res_par, const Tensor& step, const OT& ctr, const OT& att, const OT& att_hist,
               const OT& pg, const OT& pg_hist, int64_t T, int64_t Na, int64_t beam, int64_t K, int64_t stop_id,
               int64_t min_dec, int64_t max_dec) {
  chk(top_ids, I32, "top_ids"); chk(top_lp, F32, "top_lp"); chk(lp_sum, F32, "lp_sum"); chk(latest, I32, "latest");
  chk(gidx, I32, "gidx"); chk(tok_hist, I32, "tok_hist"); chk(par_hist, I32, "par_hist"); chk(done, I32, "done");
  chk(res_count, I32, "res_count"); chk(res_score, F32, "res_score"); chk(res_len, I32, "res_len");
  chk(res_step, I32, "res_step"); chk(res_par, I32, "res_par"); chk(step, I32, "step"); chko(ctr, I32, 1, "ctr");
  const int64_t R = Na * beam;
  TORCH_CHECK(beam >= 1 && beam <= 16 && K >= 1 && K <= 16 && beam * K <= 64, "bad beam args");
  numel_eq(top_ids, R * K, "top_ids"); numel_eq(top_lp, R * K, "top_lp"); numel_eq(lp_sum, R, "lp_sum");
  numel_eq(latest, R, "latest"); numel_eq(gidx, R, "gidx"); numel_eq(tok_hist, max_dec * R, "tok_hist");
  numel_eq(par_hist, max_dec * R, "par_hist"); numel_eq(done, Na, "done"); numel_eq(res_count, Na, "res_count");
  numel_eq(res_score, R, "res_score"); numel_eq(res_len, R, "res_len"); numel_eq(res_step, R, "res_step");
  numel_eq(res_par, R, "res_par"); numel_eq(step, 1, "step");
  TORCH_CHECK(att.has_value() == att_hist.has_value() && pg.has_value() == pg_hist.has_value() &&
              (!pg.has_value() || att.has_value()), "att/att_hist and pg/pg_hist come in pairs (pg needs att)");
  chko(att, F32, R * T, "att"); chko(att_hist, F32, max_dec * R * T, "att_hist");
  chko(pg, F32, R, "pg"); chko(pg_hist, F32, max_dec * R, "pg_hist");
  launch_beam_step(P<int>(top_ids), P<float>(top_lp), P<float>(lp_sum), P<int>(latest), P<int>(gidx), P<int>(tok_hist),
                   P<int>(par_hist), P<int>(done), P<int>(res_count), P<float>(res_score), P<int>(res_len),
                   P<int>(res_step), P<int>(res_par), P<int>(step), (unsigned*)PO<int>(ctr), PO<float>(att),
                   PO<float>(att_hist), PO<float>(pg), PO<float>(pg_hist), (int)T, Na, beam, K, stop_id, min_dec,
                   max_dec, stream());
}

void beam_gather(const Tensor& gidx, const Tensor& latest, const Tensor& c_src, const Tensor& h_src,
                 const Tensor& ctx_src, const Tensor& a_src, const OT& cov_src, const Tensor& XGtab, const Tensor& Xtab,
                 const Tensor& c_out, const Tensor& h_out, const Tensor& ctx_out, const Tensor& ctxb_out,
                 const OT& cov_out, const Tensor& XG_out, const Tensor& x_out, int64_t R, int64_t H, int64_t A,
                 int64_t T, int64_t E, int64_t V, int64_t unk, const OT& step) {
  chko(step, I32, 1, "step");  // optional decode-step counter advanced by this launch
  chk(gidx, I32, "gidx"); chk(latest, I32, "latest"); chk(c_src, F32, "c_src"); chk(h_src, BF, "h_src");
  chk(ctx_src, F32, "ctx_src"); chk(a_src, F32, "a_src"); chk(XGtab, F32, "XGtab"); chk(Xtab, F32, "Xtab");
  chk(c_out, F32, "c_out"); chk(h_out, BF, "h_out"); chk(ctx_out, F32, "ctx_out"); chk(ctxb_out, BF, "ctxb_out");
  chk(XG_out, F32, "XG_out"); chk(x_out, F32, "x_out");
  numel_eq(gidx, R, "gidx"); numel_eq(latest, R, "latest"); numel_eq(c_src, R * H, "c_src"); numel_eq(h_src, R * H, "h_src");
  numel_eq(ctx_src, R * A, "ctx_src"); numel_eq(a_src, R * T, "a_src"); numel_eq(XGtab, V * 4 * H, "XGtab");
  numel_eq(Xtab, V * E, "Xtab"); numel_eq(c_out, R * H, "c_out"); numel_eq(h_out, R * H, "h_out");
  numel_eq(ctx_out, R * A, "ctx_out"); numel_eq(ctxb_out, R * A, "ctxb_out"); numel_eq(XG_out, R * 4 * H, "XG_out");
  numel_eq(x_out, R * E, "x_out"); chko(cov_src, F32, R * T, "cov_src"); chko(cov_out, F32, R * T, "cov_out");
  TORCH_CHECK(unk >= 0 && unk < V, "bad unk id");
  TORCH_CHECK(!PO<float>(cov_out) || PO<float>(cov_src), "coverage gather needs cov_src");
  launch_beam_gather(P<int>(gidx), P<int>(latest), P<float>(c_src), P<bf16>(h_src), P<float>(ctx_src), P<float>(a_src),
                     PO<float>(cov_src), P<float>(XGtab), P<float>(Xtab), P<float>(c_out), P<bf16>(h_out),
                     P<float>(ctx_out), P<bf16>(ctxb_out), PO<float>(cov_out), P<float>(XG_out), P<float>(x_out), R, H,
                     A, T, E, V, unk, PO<int>(step), stream());
}

void linear2(const Tensor& a1, int64_t K1, const OT& a2, int64_t K2, const Tensor& Wt, const OT& bias, const OT& add,
             const OT& out, const OT& outb, int64_t B, int64_t N) {
  chk(a1, BF, "a1"); chk(Wt, BF, "Wt");
  TORCH_CHECK(K1 % 32 == 0 && K2 % 32 == 0 && N % 16 == 0 && K1 > 0, "linear2: K multiples of 32, N of 16");
  TORCH_CHECK((K2 == 0) == !(a2.has_value() && a2->defined()), "linear2: a2 given iff K2 > 0");
  numel_eq(a1, B * K1, "a1"); chko(a2, BF, B * K2, "a2"); numel_eq(Wt, N * (K1 + K2), "Wt");
  chko(bias, F32, N, "bias"); chko(add, F32, B * N, "add"); chko(out, F32, B * N, "out"); chko(outb, BF, B * N, "outb");
  TORCH_CHECK(PO<float>(out) || PO<bf16>(outb), "linear2 needs an output");
  launch_linear2(P<bf16>(a1), K1, PO<bf16>(a2), K2, P<bf16>(Wt), PO<float>(bias), PO<float>(add), PO<float>(out),
                 PO<bf16>(outb), B, N, stream());
}

static void linear2_check(const Tensor& a1, int64_t K1, const OT& a2, int64_t K2, const Tensor& Wt, const OT& bias,
                          const OT& add, const OT& out, const OT& outb, int64_t B, int64_t N) {
  chk(a1, BF, "a1"); chk(Wt, BF, "Wt");
  TORCH_CHECK(K1 % 32 == 0 && K2 % 32 == 0 && N % 16 == 0 && K1 > 0, "linear2: K multiples of 32, N of 16");
  TORCH_CHECK((K2 == 0) == !(a2.has_value() && a2->defined()), "linear2: a2 given iff K2 > 0");
  numel_eq(a1, B * K1, "a1"); chko(a2, BF, B * K2, "a2"); numel_eq(Wt, N * (K1 + K2), "Wt");
  chko(bias, F32, N, "bias"); chko(add, F32, B * N, "add"); chko(out, F32, B * N, "out"); chko(outb, BF, B * N, "outb");
  TORCH_CHECK(PO<float>(out) || PO<bf16>(outb), "linear2 needs an output");
}
// two independent linear2 problems over the same B rows in one launch
void linear2_pair(const Tensor& a1, int64_t K1, const OT& a2, int64_t K2, const Tensor& Wt, const OT& bias,
                  const OT& add, const OT& out, const OT& outb, int64_t N, const Tensor& c1, int64_t L1, const OT& c2,
                  int64_t L2, const Tensor& Vt, const OT& vbias, const OT& vadd, const OT& vout, const OT& voutb,
                  int64_t M, int64_t B) {
  linear2_check(a1, K1, a2, K2, Wt, bias, add, out, outb, B, N);
  linear2_check(c1, L1, c2, L2, Vt, vbias, vadd, vout, voutb, B, M);
  launch_linear2_pair(P<bf16>(a1), K1, PO<bf16>(a2), K2, P<bf16>(Wt), PO<float>(bias), PO<float>(add), PO<float>(out),
                      PO<bf16>(outb), N, P<bf16>(c1), L1, PO<bf16>(c2), L2, P<bf16>(Vt), PO<float>(vbias),
                      PO<float>(vadd), PO<float>(vout), PO<bf16>(voutb), M, B, stream());
}

void pgen(const Tensor& ctx, const Tensor& c, const Tensor& h, const Tensor& x, const Tensor& w, const Tensor& b,
          const Tensor& pg, int64_t R, int64_t A, int64_t H, int64_t E) {
  chk(ctx, F32, "ctx"); chk(c, F32, "c"); chk(h, BF, "h"); chk(x, F32, "x"); chk(w, F32, "w"); chk(b, F32, "b");
  chk(pg, F32, "pg");
  numel_eq(ctx, R * A, "ctx"); numel_eq(c, R * H, "c"); numel_eq(h, R * H, "h"); numel_eq(x, R * E, "x");
  numel_eq(w, A + 2 * H + E, "w"); numel_eq(b, 1, "b"); numel_eq(pg, R, "pg");
  launch_pgen(P<float>(ctx), P<float>(c), P<bf16>(h), P<float>(x), P<float>(w), P<float>(b), P<float>(pg), R, A, H, E,
              stream());
}

// det: one workgroup row split (each gw column summed by one thread in row order, no atomics race)
void pgen_bwd(const Tensor& ctx, const Tensor& c, const Tensor& h, const Tensor& x, const Tensor& dpre,
              const Tensor& gw, int64_t N, int64_t A, int64_t H, int64_t E, bool det) {
  chk(ctx, F32, "ctx"); chk(c, F32, "c"); chk(h, BF, "h"); chk(x, F32, "x"); chk(dpre, F32, "dpre");
  chk(gw, F32, "gw");
  numel_eq(ctx, N * A, "ctx"); numel_eq(c, N * H, "c"); numel_eq(h, N * H, "h"); numel_eq(x, N * E, "x");
  numel_eq(dpre, N, "dpre"); numel_eq(gw, A + 2 * H + E, "gw");
  (void)det;  // (the split sums are added in a fixed order in every mode)
  const int64_t Kt = A + 2 * H + E, S = pgen_bwd_splits((int)N, (int)A, (int)H, (int)E);
  auto part = at::empty({S, Kt}, gw.options());
  auto cpart = at::empty({(int64_t)colsum_det_chunks((int)S, (int)Kt), Kt}, gw.options());
  launch_pgen_bwd(P<float>(ctx), P<float>(c), P<bf16>(h), P<float>(x), P<float>(dpre), P<float>(gw), P<float>(part),
                  P<float>(cpart), N, A, H, E, stream());
}

// gb (+)= sum(dpre) with atomics: pass the zeroed p_gen bias-gradient slot (or None: the caller sums)
void pgen_dirs(const Tensor& dpre, const Tensor& w, const Tensor& dctx, const Tensor& dc, const Tensor& dh,
               const Tensor& dx, const OT& gb, int64_t N, int64_t A, int64_t H, int64_t E) {
  chk(dpre, F32, "dpre"); chk(w, F32, "w"); chk(dctx, F32, "dctx"); chk(dc, F32, "dc"); chk(dh, F32, "dh");
  chk(dx, F32, "dx"); chko(gb, F32, 1, "gb");
  numel_eq(dpre, N, "dpre"); numel_eq(w, A + 2 * H + E, "w"); numel_eq(dctx, N * A, "dctx"); numel_eq(dc, N * H, "dc");
  numel_eq(dh, N * H, "dh"); numel_eq(dx, N * E, "dx");
  launch_pgen_dirs(P<float>(dpre), P<float>(w), P<float>(dctx), P<float>(dc), P<float>(dh), P<float>(dx), PO<float>(gb),
                   (int)N, (int)A, (int)H, (int)E, stream());
}

}  // namespace

TORCH_LIBRARY(tsamd, m) {
  m.def("lstm_enc_fwd_step", &lstm_enc_fwd_step);
  m.def("lstm_enc_bwd_step", &lstm_enc_bwd_step);
  m.def("lstm_persistent_grid", &lstm_persistent_grid_op);
  m.def("lstm_persistent_capacity", &lstm_persistent_capacity_op);
  m.def("lstm_persistent_launches", &lstm_persistent_launches_op);
  m.def("rs_fwd", &rs_fwd);
  m.def("vocab_topk_pg", &vocab_topk_pg);
  m.def("rs_bwd", &rs_bwd);
  m.def("lstm_persistent_xbuf", &lstm_persistent_xbuf_op);
  m.def("lstm_fwd_persistent", &lstm_fwd_persistent);
  m.def("lstm_fwd_persistent_fx", &lstm_fwd_persistent_fx);
  m.def("lstm_persistent_fx_ok", &lstm_persistent_fx_ok_op);
  m.def("lstm_bwd_persistent", &lstm_bwd_persistent);
  m.def("attn_score", &attn_score);
  m.def("attn_softmax_ctx", &attn_softmax_ctx);
  m.def("attn_bwd_step", &attn_bwd_step);
  m.def("attn_row_ok", &attn_row_ok);
  m.def("attn_fwd_row", &attn_fwd_row);
  m.def("attn_bwd_row", &attn_bwd_row);
  m.def("attn_rowp_ok", &attn_rowp_ok);
  m.def("attn_fwd_rowp", &attn_fwd_rowp);
  m.def("attn_bwd_rowp", &attn_bwd_rowp);
  m.def("attn_bwd_feat", &attn_bwd_feat);
  m.def("attn_chunks", &attn_chunks);
  m.def("dec_cell_fwd", &dec_cell_fwd);
  m.def("dec_sproj", &dec_sproj);
  m.def("dec_bwd_cell", &dec_bwd_cell);
  m.def("dec_bwd_dz", &dec_bwd_dz);
  m.def("ptr_loss", &ptr_loss);
  m.def("wgrad_tn", &wgrad_tn);
  m.def("wgrad_tt", &wgrad_tt);
  m.def("ctx_bmm_ok", &ctx_bmm_ok_op);
  m.def("ctx_fwd", &ctx_fwd);
  m.def("ctx_da", &ctx_da);
  m.def("ctx_de", &ctx_de);
  m.def("wgrad_tt_ws", &wgrad_tt_ws);
  m.def("pgen_dirs", &pgen_dirs);
  m.def("pack_cast", &pack_cast);
  m.def("pack_max_jobs", &pack_max_jobs_op);
  m.def("pack_job_cols", &pack_job_cols_op);
  m.def("debug_enabled", &debug_enabled);
  m.def("debug_status", &debug_status);
  m.def("debug_clear", &debug_clear);
  m.def("gemm_bt_ok", &gemm_bt_ok);
  m.def("gemm_bt", &gemm_bt);
  m.def("gemm_bt_splitk_ws", &gemm_bt_splitk_ws);
  m.def("gemm_bt_splitk", &gemm_bt_splitk);
  m.def("gemm_bt_merge", &gemm_bt_merge);
  m.def("cu_hold_max_lds", &cu_hold_max_lds_op);
  m.def("cu_hold", &cu_hold);
  m.def("tanh_eval", &tanh_eval);
  m.def("tanh_tput", &tanh_tput);
  m.def("vocab_train_tiles", &vocab_train_tiles_op);
  m.def("vocab_train_fwd", &vocab_train_fwd);
  m.def("vocab_train_bwd", &vocab_train_bwd);
  m.def("emb_grad", &emb_grad);
  m.def("emb_grad_sorted", &emb_grad_sorted);
  m.def("emb_grad_det", &emb_grad_det);
  m.def("emb_grad_det_chunks", &emb_grad_det_chunks_op);
  m.def("to_step_frame", &to_step_frame);
  m.def("from_step_frame", &from_step_frame);
  m.def("transpose_bta", &transpose_bta);
  m.def("tr01", &tr01);
  m.def("linear2_pair", &linear2_pair);
  m.def("cast_colsum", &cast_colsum);
  m.def("colsum", &colsum);
  m.def("step_frame_hop", &step_frame_hop);
  m.def("ptr_rowfin", &ptr_rowfin);
  m.def("clip_adagrad", &clip_adagrad);
  m.def("opt_parts", &opt_parts);
  m.def("final_topk", &final_topk);
  m.def("topk_parts", &topk_parts);
  m.def("beam_step", &beam_step);
  m.def("beam_gather", &beam_gather);
  m.def("linear2", &linear2);
  m.def("pgen", &pgen);
  m.def("vocab_topk", &vocab_topk);
  m.def("vocab_topk_parts", &vocab_topk_parts);
  m.def("vocab_span_probe", &vocab_span_probe);
  m.def("attn_fwd_row_probe", &attn_fwd_row_probe);
  m.def("vocab_select_stamps", &vocab_select_stamps);
  m.def("lstm_bwd_stamps", &lstm_bwd_stamps);
  m.def("vocab_topk_beam", &vocab_topk_beam);
  m.def("dec_cell_fwd_beam", &dec_cell_fwd_beam);
  m.def("beam_sproj_xmerge", &beam_sproj_xmerge);
  m.def("attn_fwd_row_beam", &attn_fwd_row_beam);
  m.def("pgen_bwd", &pgen_bwd);
}
