/*
 * tik.h — C ABI of libtik.so, the MI355X-native temporal-IK engine.
 *
 * Every compute entry point takes caller-owned DEVICE pointers (fp32,
 * row-major, explicit dims) and a hipStream_t passed as `void*` (NULL = the
 * legacy default stream), is stream-ordered, and returns an int status:
 * TIK_OK (0) or a negative TIK_E_* code; tik_last_error() returns the text of
 * the calling thread's last failure. Handles own their device weights and
 * workspace; per-call functions allocate only through the handle. One
 * handle serves one stream at a time: calls on the same handle must be
 * stream-ordered (they share its workspace, which a call may grow). Distinct
 * handles are independent. An online-IK stream (tik_stream_*) owns its own
 * workspace and a reference on its model, so it may run concurrently with
 * batch calls on that model's handle, and outlives tik_model_destroy.
 *
 * Each entry point names the reference interface it replaces
 * (paths relative to the reference repository root).
 */
#ifndef TIK_H
#define TIK_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TIK_OK 0
#define TIK_E_INVALID (-1)   /* bad argument / shape: Python raises ValueError  */
#define TIK_E_HIP (-2)       /* HIP runtime error: Python raises RuntimeError   */
#define TIK_E_MISSING (-3)   /* missing state-dict tensor: Python raises KeyError */
#define TIK_E_NOMEM (-4)     /* device allocation failed                        */

typedef struct tik_model* tik_model_t;
typedef struct tik_fk* tik_fk_t;

/* One named host fp32 tensor of a state dict (weight ABI = reference keys). */
typedef struct {
    const char* name;      /* e.g. "backbone.st_gcn_networks.3.tcn.2.weight" */
    const float* data;     /* host pointer, contiguous                        */
    int ndim;
    int64_t shape[4];
} tik_tensor;

const char* tik_last_error(void);
const char* tik_version(void);
// Debug: with TIK_GUARD=1 in the environment every library buffer carries
// 1 MiB guard zones; returns the number of written guard zones (description
// in tik_last_error(), guards re-armed), or < 0 on error.
int tik_debug_check_guards(void);
// Debug: with TIK_CHECKSUM set, every launch of the IK forward is followed by
// a synchronising checksum of its output; copies "label:hex;..." of the
// launches since the last call into buf and clears the record.
int tik_debug_checksums(char* buf, int len);

/* ------------------------------------------------------------------------
 * IK model: PoseRegressor = StgGcn18 backbone + MLP head.
 * Replaces pose_trainer.py:66-133 (PoseRegressor.__init__/forward) and
 * IKPoseTrainer.forward pose_trainer.py:143-144, as called by
 * inference.run_inference inference.py:51.
 *
 * tik_model_create: `tensors` is the PoseRegressor state dict (keys without
 * the Lightning "regressor." prefix; num_batches_tracked ignored). Layer
 * shapes are inferred from the tensors (pose_trainer.py:76-83 config).
 * BatchNorm (eval) is folded into the convolutions on the host, then the
 * packed weights are uploaded once.
 * ---------------------------------------------------------------------- */
int tik_model_create(const tik_tensor* tensors, int n_tensors, tik_model_t* out);
int tik_model_destroy(tik_model_t m);
/* Output frames T' for an input window of T frames (4 stride-2 layers). */
int tik_model_out_frames(tik_model_t m, int T);
/* Grow the handle-owned workspace for batches up to (N,T); optional. */
int tik_model_reserve(tik_model_t m, int N, int T);
/* keypoints x: (N,T,V=17,C=3) fp32 device; poses: (N,T',66) fp32 device. */
int tik_ik_forward(tik_model_t m, const float* x, int N, int T, float* poses, void* stream);
/* Backbone only (StgGcn18.forward, st_gcn_aaai18.py:113-133): feat (N,T',V*Cout).
 * A handle created from a backbone-only state dict (StgGcn18's own keys, no
 * head) serves this call only; tik_ik_forward and tik_stream_create refuse it. */
int tik_backbone_forward(tik_model_t m, const float* x, int N, int T, float* feat, void* stream);

/* GEMM arithmetic (both accumulate in fp32):
 * 0 = exact fp32 MFMA (v_mfma_f32_16x16x4_f32);
 * 2 = 6-product bf16 split (v_mfma_f32_16x16x32_bf16 on x = p0 + p1 + p2,
 *     products p_i q_j with i + j <= 2: fp32's exponent range, ~2^-24
 *     relative per product) — the DEFAULT.
 * (1, a 3-term f16 split with f16's narrower range, is retired: the setters
 * return TIK_E_INVALID for it.) The environment variable
 * TIK_PRECISION=fp32|bf16x3 picks the arithmetic at handle creation. */
#define TIK_PREC_F32 0
#define TIK_PREC_BF16X3 2
int tik_model_set_precision(tik_model_t m, int prec);
int tik_model_get_precision(tik_model_t m);

/* Per-launch HIP-event profiling of the model's kernels (used by bench.py):
 * tik_model_profile(m, n) records up to n launches (0 disables, clears);
 * after synchronising, tik_model_profile_read returns launch i's label
 * ("<tile config>.<role>"), elapsed ms, and algorithmic FLOPs / bytes. */
int tik_model_profile(tik_model_t m, int max_launches);
int tik_model_profile_count(tik_model_t m);
int tik_model_profile_read(tik_model_t m, int i, char* label, int label_len, float* ms, double* flops,
                           double* bytes);

/* ------------------------------------------------------------------------
 * One StGcnBlock (st_gcn_aaai18.py:136-214, eval mode) on channels-last data.
 * x: (N,T,V,Cin) device, out: (N,T',V,Cout) device, A_eff: (V,V) device
 * (= A * edge_importance, st_gcn_aaai18.py:129), K = 1 (uniform strategy).
 * `tensors` is the block's state dict (keys "gcn.conv.weight", "tcn.0.*",
 * "tcn.2.*", "tcn.3.*", "residual.0.*", "residual.1.*").
 * residual: 0 = none (zero), 1 = module default (iden or conv per :191-204).
 * ---------------------------------------------------------------------- */
typedef struct tik_block* tik_block_t;
int tik_block_create(const tik_tensor* tensors, int n_tensors, int in_channels, int out_channels,
                     int stride, int residual, const float* A_eff_host, int V, tik_block_t* out);
int tik_block_destroy(tik_block_t b);
int tik_stgcn_block_fwd(tik_block_t b, const float* x, int N, int T, float* out, void* stream);
int tik_block_set_precision(tik_block_t b, int prec);

/* ------------------------------------------------------------------------
 * ConvTemporalGraphical.forward (gconv_origin.py:56-65), reference layout.
 * x (N,Cin,T,V), A (K,V,V), W (K*Cout, Cin, t_kernel, 1), b (K*Cout) or NULL,
 * out (N,Cout,T_out,V) with T_out = (T + 2p - d*(tk-1) - 1)/s + 1. All device.
 * ---------------------------------------------------------------------- */
int tik_gconv_fwd(const float* x, int N, int Cin, int T, int V, const float* A, int K,
                  const float* W, const float* b, int Cout, int t_kernel, int t_stride,
                  int t_padding, int t_dilation, float* out, void* stream);

/* ------------------------------------------------------------------------
 * kornia angle_axis_to_rotation_matrix (common/kornia_geometry_conversion.py:125-201):
 * aa (n,3) -> R (n,3,3), device pointers.
 * ---------------------------------------------------------------------- */
int tik_aa_to_rotmat(const float* aa, int n, float* R, void* stream);

/* ------------------------------------------------------------------------
 * Windowing (mmskeleton/datasets/data_amass.py:18-42 sample_window and
 * :221-236 InferenceDataset, relative_pose=True) on the device:
 * seq (F,V,3) -> windows (n_idx, 2h+1, V, 3) for centre frames
 * idx0 .. idx0+n_idx-1, edge-padded, root-relative (root = mean of joints
 * root_a, root_b; COCO 11/12). Returns TIK_E_INVALID when any requested
 * window would raise ValueError or be short in the reference.
 * ---------------------------------------------------------------------- */
int tik_window_gather(const float* seq, int F, int V, int idx0, int n_idx, int h, int root_a,
                      int root_b, int relative, float* windows, void* stream);

/* ------------------------------------------------------------------------
 * moveai_3d -> COCO-17 keypoints on the device (inference.py:121-133 with
 * common/keypoints_util.py:27-60 generate_moveai3d_to_coco_mappings /
 * convert_seq_keypoints): out[f][c] = joints[f][map17[c]] (map17: 17 host ints,
 * -1 = none), COCO 0 = 0.5 (joints[f][J-1] + joints[f][J-2]) (nose = mid of
 * the ears), 1 = joints[f][J-2], 2 = joints[f][J-1] (eyes = ears), then
 * (x, y, z) -> (x, z, -y). joints (F,J,3), out (F,17,3), device fp32.
 * ---------------------------------------------------------------------- */
int tik_moveai_to_coco(const float* joints, int F, int J, const int* map17_host, float* out, void* stream);

/* ------------------------------------------------------------------------
 * Online IK (BASELINE.json config #5): stride-1 sliding window over a live
 * sequence. tik_stream_push copies one frame (V=17 x 3 host floats) into a
 * device ring, gathers the window centred h = win_size/2 frames back (left
 * edge clamped as data_amass.py:18-42), runs the IK forward (N=1) and returns
 * pose row 0 (66 floats) — identical to inference.run_inference's frame
 * (inference.py:37-67). Returns 1 when a pose was produced (after h+1 pushes),
 * 0 before, <0 on error. The step is one hipGraph replay when use_graph != 0.
 * Flush the last h frames by pushing the last frame h more times.
 * ---------------------------------------------------------------------- */
/* The stream keeps a reference on `model` (released by tik_stream_destroy)
 * and a private workspace sized for (1, 2h+1): batch calls on the model handle
 * (any size, any stream) do not disturb a live stream. */
typedef struct tik_stream* tik_stream_t;
int tik_stream_create(tik_model_t model, int win_size, int use_graph, tik_stream_t* out);
int tik_stream_destroy(tik_stream_t s);
int tik_stream_reset(tik_stream_t s);
int tik_stream_push(tik_stream_t s, const float* frame_host, float* pose_host);
/* Which step the stream runs: 1 = the single dataflow kernel (online.hip:
 * only the frames pose row 0 depends on, fp32, frame read from and pose
 * written to pinned host memory by the kernel; TIK_ONLINE=0 disables it),
 * 0 = the layered IK forward on the whole window (models it cannot run). */
int tik_stream_path(tik_stream_t s);
/* Debug (TIK_ONLINE_TRACE=1 at create): the last step's per-task timestamps
 * {ticket taken, inputs ready, staged, computed, reduced, stores complete,
 * done, workgroup} (s_memrealtime ticks, 100 MHz; staged .. reduced: gcn and
 * temporal-conv tasks only)
 * in task order; returns the task count. */
int tik_debug_stream_trace(tik_stream_t s, long long* out, int cap);
/* Test hook: mark the dataflow kernel's dependency-timeout flag, as a real
 * 0.5 s wait timeout would; the next tik_stream_push then fails (that frame's
 * pose is invalid, the frame is still appended) and the one after it works. */
int tik_debug_stream_inject_error(tik_stream_t s);
/* Test hook: move the stream's frame count to `count`, which must be congruent to
 * the current count modulo 2 * (2h + 1) (the same ring slot and launch parity),
 * e.g. to just below the 2^30 wrap of stream_next_count (csrc/online.h). */
int tik_debug_stream_set_count(tik_stream_t s, int count);

/* ------------------------------------------------------------------------
 * Training-data generation (data half): AmassDataset
 * (mmskeleton/datasets/data_amass.py:87-218) on the GPU.
 * tik_rotate_root_z: regenerate_data's root-orientation augmentation
 * (:184-190) in place on pose rows (ld floats, first 3 = root axis-angle):
 * rotvec(R_z(angle) R(root)), float64 as scipy's Rotation does it.
 * tik_train_windows: __getitem__ (:125-154) for B items: edge-padded window
 * (2h+1 frames, h <= 64) of the FK joints [rows][n_joints][3] -> COCO-17
 * (coco_map, host) -> root-relative -> per-joint Gaussian noise (sigma, host:
 * coco_kps_sigma) -> windows [B][2h+1][17][3]; target = pose row of the
 * window's last frame, first 66 values -> [B][66]. Items (device int arrays):
 * sequence start row, sequence length, window centre, dataset index (the
 * noise stream: counter-based, keyed by (seed, index)). The caller checks the
 * reference's ValueError / short-window cases (the Python layer does).
 * ---------------------------------------------------------------------- */
int tik_rotate_root_z(float* poses, int F, int ld, double angle, void* stream);
int tik_train_windows(const float* joints, int n_joints, const float* poses, int pose_ld, const int* item_start,
                      const int* item_len, const int* item_idx, const int* item_uid, int B, int h,
                      const int* coco_map, const float* sigma, int relative, int add_noise, unsigned long long seed,
                      float* windows, float* target, void* stream);

/* ------------------------------------------------------------------------
 * Training step (optimizer half). Replaces
 * IKPoseTrainer.training_step (pose_trainer.py:146-155) as Lightning runs it:
 * train-mode forward (batch-statistics BatchNorm with the running-stat
 * update, Dropout(0.7) in the head, pose_trainer.py:89-92), nn.MSELoss
 * against the target poses (PoseLosses, :42-50), backward, and one
 * torch.optim.Adam(lr) update (configure_optimizers, :196-197).
 *
 * tik_trainer_create: the PoseRegressor state dict (as tik_model_create,
 *   incl. "tik.strides"); parameters and buffers are copied to the device.
 * tik_trainer_step: x [N][T][17][3], target [N][T'][66] (device fp32);
 *   dropout_mask [N*T'][512] of 0/1 (device), or NULL = a counter-based mask
 *   keyed by `seed`; loss: device float (or NULL). Stream-ordered.
 * tik_trainer_count / _tensor / _read: the state dict after the last step,
 *   in the reference's names and layouts (kind 0 = parameter, 1 = buffer);
 *   what = 0 value, 1 last gradient, 2 Adam exp_avg, 3 Adam exp_avg_sq,
 *   copied to a device pointer. tik_trainer_steps: updates taken
 *   (BatchNorm num_batches_tracked).
 * ---------------------------------------------------------------------- */
typedef struct tik_trainer* tik_trainer_t;
int tik_trainer_create(const tik_tensor* tensors, int n_tensors, float lr, tik_trainer_t* out);
int tik_trainer_destroy(tik_trainer_t t);
int tik_trainer_step(tik_trainer_t t, const float* x, int N, int T, const float* target, const float* dropout_mask,
                     unsigned long long seed, float* loss, void* stream);
int tik_trainer_out_frames(tik_trainer_t t, int T);
int tik_trainer_count(tik_trainer_t t);
int tik_trainer_tensor(tik_trainer_t t, int i, char* name, int name_len, int64_t* shape4, int* ndim, int* kind);
int tik_trainer_read(tik_trainer_t t, int i, int what, float* dst, void* stream);
long long tik_trainer_steps(tik_trainer_t t);
/* Debug / test hook: the last step's saved activations of block `layer`
 * (which 0 output, 2 tcn conv output, 3 post-ReLU tcn input, 4 graph-mix
 * output, 5 gcn conv output; 6 the head's first Linear output), and with
 * TIK_TRAIN_DEBUG=1 (TIK_TRAIN_DEBUG_LAYER=l) its input gradient (1) and
 * backward intermediates (10..14); n floats to device dst. */
int tik_trainer_debug(tik_trainer_t t, int which, int layer, float* dst, long long n, void* stream);

/* ------------------------------------------------------------------------
 * SMPL-X forward kinematics + linear blend skinning (the FK check).
 * Replaces common/smpl_util.py:8-82 (load_smplx_models / run_smpl_inference)
 * and the third-party smplx.SMPLX.forward it calls (smpl_util.py:67-69;
 * create(model_type='smplx', use_pca=False, use_face_contour=True)).
 *
 * tik_fk_create: named host tensors (integer tables passed as exact floats):
 *   v_template (V,3), shapedirs (V,3,nb), [exprdirs (V,3,ne)], posedirs (486,3V),
 *   J_regressor (55,V), lbs_weights (V,55), parents (55), faces (F,3),
 *   lmk_faces_idx (L), lmk_bary_coords (L,3), extra_verts (21),
 *   [pose_mean (55,3)] (flat_hand_mean=False hand mean),
 *   [dynamic_lmk_faces_idx (79,D), dynamic_lmk_bary_coords (79,D,3)].
 * flags bit 0: use_face_contour (needs the dynamic tables).
 * tik_fk_forward: full_pose (B,55,3) [global, 21 body, jaw, leye, reye,
 *   15 lhand, 15 rhand], betas (B,nb)/NULL, expression (B,ne)/NULL,
 *   transl (B,3)/NULL -> joints (B, 55+21+L+D, 3), verts (B,V,3) or NULL.
 * ---------------------------------------------------------------------- */
int tik_fk_create(const tik_tensor* tensors, int n_tensors, int flags, tik_fk_t* out);
int tik_fk_destroy(tik_fk_t fk);
int tik_fk_set_precision(tik_fk_t fk, int prec);
int tik_fk_num_joints(tik_fk_t fk);
int tik_fk_num_verts(tik_fk_t fk);
int tik_fk_reserve(tik_fk_t fk, int B);
int tik_fk_forward(tik_fk_t fk, const float* full_pose, const float* betas, const float* expression,
                   const float* transl, int B, float* joints, float* verts, void* stream);
/* Per-launch HIP-event profile of tik_fk_forward (fk_chain, fk_blend, fk_skin,
 * fk_landmarks), as tik_model_profile / _count / _read. */
int tik_fk_profile(tik_fk_t fk, int max_launches);
int tik_fk_profile_count(tik_fk_t fk);
int tik_fk_profile_read(tik_fk_t fk, int i, char* label, int label_len, float* ms, double* flops, double* bytes);

#ifdef __cplusplus
}
#endif
#endif /* TIK_H */
