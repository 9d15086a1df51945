// Schema definitions of the sftamd custom-op library. Implementations live next to their
// kernels (TORCH_LIBRARY_IMPL(sftamd, CUDA, ...) in each .hip file); the CPU path of every
// op is the PyTorch reference in llm_fine_tune_distributed_amd/ops/reference.py, except the
// native data-pipeline ops below which are CPU kernels.
#include <torch/library.h>

#include <string>
#include <vector>

namespace sftamd {
// csrc/ipc_allreduce.hip: one-shot peer-memory all-reduce for small messages
int64_t ipc_ar_create(int64_t cap, int64_t world, int64_t rank);
std::vector<int64_t> ipc_ar_handle(int64_t id);
void ipc_ar_open(int64_t id, std::vector<int64_t> handles);
int64_t ipc_ar_check(int64_t id);
int64_t ipc_ar_poll(int64_t id);
int64_t ipc_ar_uncached(int64_t id);
void ipc_ar_destroy(int64_t id);
// csrc/ddp_reducer.cpp: bucket planner + ready tracker of the DDP engine
std::vector<int64_t> ddp_plan(std::vector<int64_t> sizes, std::vector<int64_t> region, int64_t tied, int64_t align,
                              int64_t pad_unit, int64_t cap, int64_t first_cap, int64_t split_at);
int64_t ddp_tracker_create(std::vector<int64_t> owner_ptr, std::vector<int64_t> owners, int64_t n_buckets);
void ddp_tracker_reset(int64_t id);
std::vector<int64_t> ddp_tracker_mark(int64_t id, int64_t param);
std::vector<int64_t> ddp_tracker_drain(int64_t id);
std::vector<int64_t> ddp_tracker_pending(int64_t id);
void ddp_tracker_destroy(int64_t id);
// csrc/dispatch_trace.cpp
void dispatch_trace(bool on);
std::string dispatch_trace_read();
int64_t set_cu_budget(int64_t n);
}

TORCH_LIBRARY(sftamd, m) {
  // runtime: CU-restricted HIP stream for the optimizer's side stream (no tensor arguments: catch-all kernel)
  // runtime: IPC peer-memory all-reduce contexts (no tensor arguments: catch-all kernels)
  m.def("ipc_ar_create(int cap, int world, int rank) -> int", &sftamd::ipc_ar_create);
  m.def("ipc_ar_handle(int ctx) -> int[]", &sftamd::ipc_ar_handle);
  m.def("ipc_ar_open(int ctx, int[] handles) -> ()", &sftamd::ipc_ar_open);
  m.def("ipc_ar_check(int ctx) -> int", &sftamd::ipc_ar_check);
  m.def("ipc_ar_poll(int ctx) -> int", &sftamd::ipc_ar_poll);
  m.def("ipc_ar_uncached(int ctx) -> int", &sftamd::ipc_ar_uncached);
  m.def("ipc_ar_destroy(int ctx) -> ()", &sftamd::ipc_ar_destroy);
  // runtime: DDP bucket planner / ready tracker (CPU, no tensor arguments)
  m.def("ddp_plan(int[] sizes, int[] region, int tied, int align, int pad_unit, int cap, int first_cap, "
        "int split_at) -> int[]", &sftamd::ddp_plan);
  m.def("ddp_tracker_create(int[] owner_ptr, int[] owners, int n_buckets) -> int", &sftamd::ddp_tracker_create);
  m.def("ddp_tracker_reset(int id) -> ()", &sftamd::ddp_tracker_reset);
  m.def("ddp_tracker_mark(int id, int param) -> int[]", &sftamd::ddp_tracker_mark);
  m.def("ddp_tracker_drain(int id) -> int[]", &sftamd::ddp_tracker_drain);
  m.def("ddp_tracker_pending(int id) -> int[]", &sftamd::ddp_tracker_pending);
  m.def("ddp_tracker_destroy(int id) -> ()", &sftamd::ddp_tracker_destroy);
  m.def("ipc_ar_allreduce(Tensor(a!) x, int ctx, int round, int blocks=16) -> ()");
  // runtime: dispatch trace of the kernel variants launched (tests assert the default paths)
  m.def("dispatch_trace(bool on) -> ()", &sftamd::dispatch_trace);
  m.def("dispatch_trace_read() -> str", &sftamd::dispatch_trace_read);
  m.def("set_cu_budget(int n) -> int", &sftamd::set_cu_budget);
  // norms / elementwise
  m.def("rmsnorm_fwd(Tensor x, Tensor? residual, Tensor weight, float eps, int y_ld=0) -> (Tensor, Tensor, Tensor)");
  m.def("rmsnorm_bwd(Tensor dy, Tensor h, Tensor weight, Tensor rstd, Tensor? dres, Tensor(a!)? dw_out=None, bool accumulate=False) -> (Tensor, Tensor)");
  m.def("swiglu_fwd(Tensor gate_up) -> Tensor");
  m.def("cu_hog(Tensor(a!) sink, int blocks, float usec) -> ()");
  m.def("swiglu_bwd(Tensor dy, Tensor gate_up) -> Tensor");
  m.def("rope_(Tensor(a!) qkv, Tensor cos, Tensor sin, int n_q, int n_kv, int head_dim, bool inverse) -> ()");
  m.def("embedding_fwd(Tensor ids, Tensor weight) -> Tensor");
  m.def("dropout_add(Tensor? a, Tensor b, float p, int seed) -> Tensor");
  m.def("lora_widen(Tensor x, int R, float p, int seed) -> (Tensor, Tensor)");
  m.def("lora_fwd(Tensor x, Tensor A, float s, float p, int seed, int ldX=0, bool save_xd=False, bool swiglu=False) -> (Tensor, Tensor)");
  m.def("lora_bwd_dx(Tensor base, Tensor dxa, Tensor A, float p, int seed, Tensor? gu=None) -> Tensor");
  m.def("lora_tsum(Tensor X, int K, Tensor S, float p, int seed) -> Tensor");
  m.def("lora_fwd_inplace(Tensor(a!) X, int K, Tensor A, float s, float p, int seed) -> ()");
  m.def("lora_dxa(Tensor dy, Tensor Bc, float s) -> Tensor");
  m.def("lora_dxa_blocks(Tensor dy, Tensor Bc, int[] o, int[] rows, int[] c, int r, float s) -> Tensor");
  m.def("lora_grad_out(Tensor sum, Tensor(a!)[] outs, int[] r0, int[] c0, bool tr, int[] accumulate) -> ()");
  m.def("lora_grad_out2(Tensor sa, Tensor(a!)[] oa, int[] ra, int[] ca, bool ta, int[] aa, Tensor sb, "
        "Tensor(b!)[] ob, int[] rb, int[] cb, bool tb, int[] ab) -> ()");
  m.def("copy2d_batch(Tensor desc, int max_elems) -> ()");
  m.def("embedding_bwd(Tensor dy, Tensor sorted_ids, Tensor perm, Tensor(a!) grad_weight) -> ()");
  // loss
  m.def("ce_fwd(Tensor(a!) logits, Tensor labels, Tensor inv_count, bool write_grad) -> Tensor");
  // attention
  m.def("flash_fwd(Tensor qkv, Tensor cu_seqlens, int max_seqlen, int n_q, int n_kv, int head_dim, float scale, bool causal) -> (Tensor, Tensor)");
  m.def("flash_bwd(Tensor dout, Tensor qkv, Tensor out, Tensor lse, Tensor cu_seqlens, int max_seqlen, int n_q, int n_kv, int head_dim, float scale, bool causal, Tensor? delta=None) -> Tensor");
  m.def("flash_bwd_rope(Tensor dout, Tensor qkv, Tensor out, Tensor lse, Tensor cu_seqlens, int max_seqlen, int n_q, int n_kv, int head_dim, float scale, bool causal, Tensor cos, Tensor sin, Tensor? delta=None) -> Tensor");
  m.def("decode_attention(Tensor q, Tensor kcache, Tensor vcache, Tensor cache_len, int n_q, int n_kv, float scale) -> Tensor");
  // fused decode sampler: penalty -> temperature -> top-k -> top-p -> draw, device-resident state
  m.def("sample_token(Tensor logits, Tensor(a!) presence, Tensor(b!) state, Tensor(c!)? tok_out, Tensor(d!)? pos_out, Tensor(e!)? len_out, Tensor(f!)? log, float temperature, int top_k, float top_p, float repetition_penalty, bool do_sample, int seed) -> ()");
  // weight-gradient GEMM: out[N,K] (+)= dy[T,N]^T x[T,K]
  m.def("wgrad_gemm(Tensor(a!) out, Tensor dy, Tensor x, bool accumulate, int cfg=14, Tensor(b!)? norm=None) -> ()");
  m.def("wgrad_gemm_multi(Tensor(a!)[] outs, Tensor[] dys, Tensor[] xs, int[] accs, Tensor(b!)[] norms, int split_all=0, int split_left=0) -> ()");
  m.def("wgrad_gemm_pair(Tensor(a!) out0, Tensor dy0, Tensor x0, bool acc0, Tensor(b!)? norm0, Tensor(c!) out1, Tensor dy1, Tensor x1, bool acc1, Tensor(d!)? norm1, int split_all=0) -> ()");
  // input-gradient GEMM dX = dy w (w [K, N]), optional fused SwiGLU backward (csrc/gemm_dgrad.hip)
  m.def("dgrad_gemm(Tensor dy, Tensor w, Tensor? gate_up=None, int cfg=14) -> Tensor");
  m.def("dgrad_gemm_delta(Tensor dy, Tensor w, Tensor attn_out) -> (Tensor, Tensor)");
  // forward-layout GEMM C = a w^T with fused epilogues (csrc/gemm_tn.hip)
  m.def("gemm_tn(Tensor a, Tensor w, int cfg=0) -> Tensor");
  m.def("gemm_tn_swiglu(Tensor x, Tensor w_gate_up, int cfg=5) -> (Tensor, Tensor)");
  m.def("gemm_tn_rope(Tensor x, Tensor w, Tensor cos, Tensor sin, int rope_cols, int cfg=0) -> Tensor");
  // optimizer
  m.def("sumsq(Tensor x) -> Tensor");
  m.def("sumsq_chunks(Tensor x, Tensor chunks) -> Tensor");
  m.def("adamw_flat(Tensor(a!) param, Tensor grad, Tensor(b!)? master, Tensor(c!) exp_avg, Tensor(d!) exp_avg_sq, Tensor clip_coef, float lr, float beta1, float beta2, float eps, float weight_decay, float bc1, float bc2, int sr_seed=0, int sr_offset=0) -> ()");
  // native data pipeline (CPU)
  m.def("pack_sequences(Tensor tokens, Tensor offsets, Tensor order, int max_tokens, int pad_id, int pad_multiple) -> (Tensor, Tensor, Tensor, Tensor, Tensor)");
  m.def("pad_batch(Tensor tokens, Tensor offsets, Tensor order, int pad_id, int pad_multiple, int max_length) -> (Tensor, Tensor, Tensor)");
}
