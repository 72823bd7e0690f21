// Host launch entry points of the gfx950 kernels (implemented in *.hip, called from bindings.cpp).
#pragma once
#include <hip/hip_runtime.h>
typedef __bf16 bf16;

void launch_lstm_enc_fwd_step(const float* gx, const float* bias, const bf16* Wt, bf16* hs, float* cs, float* acts, bf16* out,
                              const int* lens, int s, int T, int B, int H, hipStream_t st);
void launch_lstm_enc_bwd_step(bf16* dz, const bf16* Wn, const float* dout, const float* dh_fin, float* dc_carry,
                              const float* acts, const float* cs, const int* lens, int s, int T, int B, int H,
                              hipStream_t st);

void launch_attn_score(const bf16* F, const float* s, const float* v, const float* wc, const float* cov,
                       const int* lens, float* e, int B, int T, int A, int rep, hipStream_t st);
void launch_attn_softmax_ctx(const float* e, const bf16* E, const int* lens, const float* cov, float* a_out,
                             float* cov_out, float* covloss, float* ctx, bf16* ctx_bf, int B, int T, int A, int rep,
                             hipStream_t st);
int attn_nchunk(int T);
void launch_attn_bwd_step(const bf16* E, const bf16* F, const float* s, const float* v, const float* wc,
                          const float* cov, const float* a, const float* dctx, const float* ctx, const float* Ga,
                          const float* dcov_next, const float* gcl, const int* lens, float* de_out, float* ds,
                          float* dcov_out, int B, int T, int A, hipStream_t st);
void launch_attn_bwd_feat(const bf16* F, const float* S_all, const float* v, const float* wc, const float* cov_all,
                          const float* de_all, const int* lens, bf16* dF, float* dv, float* dwc, int D, int B, int T,
                          int A, int nslot, hipStream_t st, const int* dlen = nullptr);

bool attn_row_supported(int A, int T);
void launch_attn_fwd_row_probe(const bf16* F, const bf16* E, const float* s, const float* v, const float* wc,
                               const float* cov, const int* lens, float* a_out, float* ctx, int B, int T, int rep,
                               int probe, hipStream_t st);
void launch_attn_fwd_row(const bf16* F, const bf16* E, const float* s, const float* v, const float* wc,
                         const float* cov, const int* lens, float* a_out, float* cov_out, float* covloss, float* ctx,
                         bf16* ctx_bf, int B, int T, int A, int rep, hipStream_t st, const int* cg = nullptr,
                         const float* asrc = nullptr, float* cov_keep = nullptr);
void launch_attn_bwd_row(const bf16* E, const bf16* F, const float* s, const float* v, const float* wc,
                         const float* cov, const float* a, const float* dctx, const float* ctx, const float* Ga,
                         const float* dcov_next, const float* gcl, const int* lens, float* de_out, float* ds,
                         float* dcov_out, int B, int T, int A, hipStream_t st);

bool attn_rowp_supported(int A, int T, int EG);
void launch_attn_fwd_rowp(const bf16* F, const bf16* G, const float* s, const float* v, const float* wc,
                          const float* cov, const int* lens, float* a_out, float* cov_out, float* covloss, float* gx,
                          bf16* gx_bf, int B, int T, int A, const int* dlen, int step, hipStream_t st,
                          bf16* a_bf = nullptr);
void launch_attn_bwd_rowp(const bf16* G, const bf16* F, const float* s, const float* v, const float* wc,
                          const float* cov, const float* a, const float* dx, const float* gv, const float* Ga,
                          const float* dcov_next, const float* gcl, const int* lens, float* de_out, float* ds,
                          float* dcov_out, int B, int T, int A, const int* dlen, int step, hipStream_t st);

void launch_dec_cell_fwd(const float* XG, const bf16* ctxp, const bf16* hprev, const float* cprev, const bf16* WcT,
                         float* c_out, bf16* cb_out, bf16* hb_out, float* act, int B, int H, int A, const int* dlen,
                         int step, hipStream_t st);
void launch_dec_cell_fwd_beam(const int* gidx, const int* latest, const float* XGtab, const bf16* ctxp,
                              const bf16* hprev, const float* cprev, const bf16* WcT, float* c_out, bf16* cb_out,
                              bf16* hb_out, int* step, int B, int H, int A, int V, int unk, hipStream_t st);
void launch_beam_sproj_xmerge(const bf16* cb, const bf16* hb, const bf16* WsT, const float* bs, float* s_out,
                              const bf16* ctx_src, const bf16* WicT, const float* Xtab, const int* gidx,
                              const int* latest, float* x_out, int B, int H, int A, int E, int V, int unk,
                              hipStream_t st);
void launch_dec_sproj(const bf16* cb, const bf16* hb, const bf16* WsT, const float* bs, float* s_out, int B, int H,
                      int A, const int* dlen, int step, hipStream_t st);
void launch_dec_bwd_cell(const float* ds, const bf16* Ws, const float* dC_dir, const float* dH_dir,
                         const float* dh_rec, float* dc_carry, const float* act, const float* c_now,
                         const float* c_prev, bf16* dz, int B, int H, int A, const int* dlen, int step,
                         hipStream_t st);
void launch_dec_bwd_dz(const bf16* dz, const bf16* Wbig, const float* dX_dir, const float* dCTX_dir_prev,
                       float* dx_out, float* dctx_prev_out, float* dh_rec, int B, int E, int H, int A,
                       const int* dlen, int step, hipStream_t st);

void launch_ptr_loss_bf16(const bf16* logits, const int* target, const float* rowg, const float* pgen,
                          const float* attn, const int* ext, const int* lens, float* loss_row, bf16* dlogits,
                          float* dpre, float* dA, int N, int B, int T, int V, hipStream_t st);
int ptr_loss_bf16_max_vocab();
void launch_ptr_loss(const float* logits, const float* bias, const int* target, const float* rowg, const float* pgen, const float* attn,
                     const int* ext, const int* lens, float* loss_row, bf16* dlogits, float* dpre, float* dA, int N,
                     int B, int T, int V, hipStream_t st);

void launch_clip_adagrad(float* w, float* acc, const float* g, long n, float* part, float lr, float max_norm,
                         float gscale, float* norm_out, int* flag, const int* skip, hipStream_t st);
int opt_nparts();

void launch_final_topk(const float* logits, const float* bias, const float* pgen, const float* attn, const int* ext,
                       const int* lens, int* out_ids, float* out_lp, float* part_ms, float* part_v, int* part_i, int R,
                       int V, int T, int K, int beam, hipStream_t st);
int topk_split(int V);
void launch_beam_step(const int* top_ids, const float* top_lp, float* lp_sum, int* latest, int* gidx, int* tok_hist,
                      int* par_hist, int* done, int* res_count, float* res_score, int* res_len, int* res_step,
                      int* res_par, int* step, unsigned* ctr, const float* att, float* att_hist, const float* pg,
                      float* pg_hist, int T, int Na, int beam, int K, int stop_id, int min_dec, int max_dec,
                      hipStream_t st);
void launch_beam_gather(const int* gidx, const int* latest, const float* c_src, const bf16* h_src,
                        const float* ctx_src, const float* a_src, const float* cov_src, const float* XGtab,
                        const float* Xtab, float* c_out, bf16* h_out, float* ctx_out, bf16* ctxb_out, float* cov_out,
                        float* XG_out, float* x_out, int R, int H, int A, int T, int E, int V, int unk,
                        int* step, hipStream_t st);
void launch_linear2(const bf16* a1, int K1, const bf16* a2, int K2, const bf16* Wt, const float* bias,
                    const float* add, float* out, bf16* outb, int B, int N, hipStream_t st);
void launch_linear2_pair(const bf16* a1, int K1, const bf16* a2, int K2, const bf16* Wt, const float* bias,
                         const float* add, float* out, bf16* outb, int N, const bf16* c1, int L1, const bf16* c2,
                         int L2, const bf16* Vt, const float* vbias, const float* vadd, float* vout, bf16* voutb,
                         int M, int B, hipStream_t st);
void launch_pgen(const float* ctx, const float* c, const bf16* h, const float* x, const float* w, const float* b,
                 float* pg, int R, int A, int H, int E, hipStream_t st);
int pgen_bwd_splits(int N, int A, int H, int E);
void launch_pgen_bwd(const float* ctx, const float* c, const bf16* h, const float* x, const float* dpre, float* gw,
                     float* part, float* cpart, int N, int A, int H, int E, hipStream_t st);
int lstm_persistent_grid(int H, int B);
int lstm_persistent_capacity(int H);
int lstm_persistent_launches(int H, int B);
size_t lstm_persistent_xbuf_elems(int H, int B, bool bwd);
void launch_lstm_fwd_persistent(const float* gx, const float* bias, const bf16* Wt, bf16* hs, float* cs, float* acts,
                                bf16* out, const int* lens, unsigned long long* xbuf, unsigned* err, int T, int B,
                                int H, hipStream_t st, const bf16* xsf = nullptr, const bf16* Wx0 = nullptr,
                                const bf16* Wx1 = nullptr);
bool lstm_persistent_fx_ok(int H, int B, int E);
void launch_lstm_bwd_persistent(bf16* dz, const bf16* Wn, const float* dout, const float* dh_fin, float* dc_carry,
                                const float* acts, const float* cs, const int* lens, unsigned long long* xbuf,
                                unsigned* err, float* dbias, int T, int B, int H, bool dout_bf, hipStream_t st,
                                bool dout_bf16 = false);
int vocab_topk_tiles(int V, int H);
void set_vocab_select_stamps(unsigned long long* buf);
void launch_vocab_span_probe(const bf16* X, const bf16* WT, const float* bias, float* logits, float* part_ms, int R, int V,
                             int probe, hipStream_t st);


// Beam bookkeeping fused into the vocab select kernel (the last row workgroup of each article
// runs it): lp_sum == nullptr disables it
struct BeamTail {
  float* lp_sum; int* latest; int* gidx; int* tok_hist; int* par_hist; int* done; int* res_count;
  float* res_score; int* res_len; int* res_step; int* res_par; int* step;
  unsigned* art_ctr;  // [Na] arrival counters (zeroed; reset by the last arrival)
  unsigned long long* gran;  // [R][K] candidate granules {step tag | id, log-prob} (zeroed per batch)
  int* err;           // poll-timeout flag
  const float* att; float* att_hist; const float* pg; float* pg_hist;
  int T, Na, beam, K, stop_id, min_dec, max_dec;
};
// p_gen inputs computed inside the vocab select kernel (w == nullptr: p_gen given instead)
struct PgIn {
  const float* ctx; const float* c; const bf16* h; const float* x; const float* w; const float* b; float* out;
  int A, H, E;
};
void launch_vocab_topk(const bf16* X, const bf16* WT, const float* bias, const float* pgen, const float* attn,
                       const int* ext, const int* lens, int* out_ids, float* out_lp, float* logits, float* part_ms,
                       int R, int V, int H, int T, int K, int beam, PgIn pgi, hipStream_t st,
                       const BeamTail* bt = nullptr);
int vocab_train_tiles(int V, int H);
void launch_vocab_train_fwd(const bf16* X, int ldx, const bf16* WT, const float* bias, const int* target, float* part,
                            float* zg, float* lse, float* pv, int N, int V, int H, const int* vblk, const int* vblk_n,
                            hipStream_t st);
void launch_vocab_train_bwd(const bf16* X, int ldx, const bf16* WT, const float* bias, const int* target,
                            const float* lse, const float* alpha, bf16* dl, int ldd, float* dbias, int N, int V, int H,
                            const int* vblk, const int* vblk_n, const int* vlive, int* vstate, hipStream_t st);
void launch_ptr_rowfin(const float* pv, const int* target, const float* rowg, const float* pgen, const float* attn,
                       const int* ext, const int* lens, float* loss_row, float* alpha, float* dpre, float* dA, int N,
                       int B, int T, hipStream_t st);

// reduce_states.hip
void launch_rs_fwd(const float* c_fw, const bf16* h_fw, size_t dstride, const bf16* RCt, const bf16* RHt,
                   const float* bc, const float* bh, float* pre_c, float* pre_h, float* c0, bf16* c0b, bf16* h0b,
                   bf16* cat_c, bf16* cat_h, int B, int H, hipStream_t st);
void launch_rs_bwd(const float* gc, const float* gh, const float* pre_c, const float* pre_h, const bf16* RC,
                   const bf16* RH, bf16* dpc, bf16* dph, float* gbc, float* gbh, float* dold_c, float* dold_h,
                   size_t dstride, int B, int H, hipStream_t st);

// embedding.hip
void launch_emb_grad(float* gemb, const int64_t* ids0, const float* src0, int n0, const int64_t* ids1,
                     const float* src1, int n1, int E, int V, hipStream_t st);

// frames.hip
void launch_to_step_frame(const void* src, int es, const int64_t* ids, const int64_t* rev, void* out, int B, int T,
                          int W, int S, int doff, long nsrc, hipStream_t st);
void launch_from_step_frame(const float* in, const int64_t* rev, float* out, int B, int T, int W, hipStream_t st);
void launch_step_frame_hop(const float* in, const int64_t* rev, float* out, int B, int T, int H, hipStream_t st);
void launch_transpose_bta(const bf16* in, bf16* out, int B, int T, int A, hipStream_t st);
void launch_tr01(const float* in, float* out, bf16* outb, int P, int Q, int R, bool acc, hipStream_t st);
int cast_colsum_blocks(int N, int C);
void launch_cast_colsum(const float* x, bf16* xb, float* part, float* colsum, int N, int C, hipStream_t st);
int colsum_det_chunks(int N, int C);
void launch_colsum_det(const void* x, bool bf, float* part, float* out, int N, int C, bool acc, hipStream_t st);
void launch_emb_grad_sorted(float* gemb, const int* sid, const int* perm, const float* src0, int n0,
                            const float* src1, int n1, int E, int V, hipStream_t st);
int emb_grad_det_chunks(int n);
void launch_emb_grad_det(float* gemb, const int* sid, const int* perm, const float* src0, int n0, const float* src1,
                         int n1, int E, int V, float* pf, float* pl, hipStream_t st);

// debug build record (debug.hip, dcheck.h)
int tsamd_debug_enabled();
void tsamd_debug_read(unsigned* out4);
void tsamd_debug_clear();

// weight-gradient GEMM out[M][N] += a[K][M]^T b[K][N] (wgrad.hip; out pre-zeroed, M, N % 128 == 0)
int wgrad_tn_splits(int M, int N, int K);
int wgrad_tt_splits(int M, int N, int K);
bool wgrad_tt_ok(int M, int N, int K);
void launch_wgrad_tt(const bf16* a, int lda, const bf16* b, int ldb, float* slab, float* out, int ldo, int M, int N,
                     int K, bool trans, bool acc, int nv, hipStream_t st);
bool wgrad_tt_direct(int M, int N, int K, bool trans, bool acc);
void launch_wgrad_tn(const bf16* a, int lda, const bf16* b, int ldb, float* out, int ldo, int M, int N, int K,
                     hipStream_t st);

// weight repack as one launch over a job table (pack.hip)
int pack_max_jobs();
int pack_job_cols();
void launch_pack_cast(const long* jobs, int nj, long total, hipStream_t st);

// p_gen gradient into the decoder inputs' direct terms + bias gradient (decoder.hip)
void launch_pgen_dirs(const float* dpre, const float* w, float* dctx, float* dc, float* dh, float* dx, float* gb,
                      int N, int A, int H, int E, hipStream_t st);

// probes.hip: CU hold (RCCL co-residency stand-in), device tanh accuracy / issue-rate probes
int cu_hold_max_lds();
void launch_cu_hold(int grid, unsigned long long ticks, long long* times, int lds_bytes, hipStream_t st);
void launch_tanh_eval(const float* x, float* t, float* s2, int n, int mode, hipStream_t st);
void launch_tanh_tput(const float* in, float* out, int threads, int iters, int mode, hipStream_t st);

// gemm_mfma.hip: C (+)= A[arow(m)] . Bt^T (+ bias); amode 0 plain rows, 1 step-frame gather
bool gemm_bt_supported(int M, int N, int K, int BN);
int gemm_bt_splits(int M, int N, int K);
void launch_gemm_bt_splitk(const bf16* A, long lda, const bf16* Bt, long ldb, float* slab, float* out, long ldo, int M,
                           int N, int K, bool acc, hipStream_t st);
void launch_slab_sum(const float* slab, float* out, int ldo, int M, int N, int S, bool acc, hipStream_t st);
void launch_gemm_bt(const bf16* A, long lda, const bf16* Bt, long ldb, void* C, long ldc, bool out_bf16, bool beta,
                    const float* bias, int M, int N, int K, int amode, const int64_t* ids, const int64_t* rev,
                    bf16* xsf, long nsrc, int B, int T, int dir, hipStream_t st);

// batched attention-context GEMMs (ctx_bmm.hip)
bool ctx_bmm_ok(int B, int T, int D, int A);
void launch_ctx_fwd(const bf16* att, const bf16* enc, float* ctx, bf16* ctxb, int B, int T, int D, int A, hipStream_t st);
void launch_ctx_da(const bf16* dctx, const bf16* enc, float* da, int B, int T, int D, int A, bool acc, hipStream_t st);
void launch_ctx_de(const bf16* att, const bf16* dctx, float* de, bf16* deb, int B, int T, int D, int A, hipStream_t st);

// attribution: per-phase s_memtime sums of the 32-row H = 512 BPTT (nullptr: off)
void set_lstm_bwd_stamps(unsigned long long* buf);
