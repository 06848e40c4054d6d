"""ctypes binding of librvc_amd.so (include/rvc_amd.h).

The library is built in-tree (``rvc-maker_amd/lib/librvc_amd.so``) by
``__graft_entry__.build()`` / ``make -C rvc-maker_amd/csrc``.  There is no
fallback: if the library is missing or a call fails, a RuntimeError is raised.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_double, c_float, c_int, c_int64, c_uint64, c_void_p

LIB_PATH = os.environ.get("RVC_AMD_LIB") or os.path.join(
    os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib", "librvc_amd.so")

ACT_NONE, ACT_LRELU, ACT_RELU, ACT_TANH, ACT_GELU, ACT_SIGMOID, ACT_LOGCLAMP = 0, 1, 2, 3, 4, 5, 6


class Conv1dArgs(ctypes.Structure):
    _fields_ = [("x", c_void_p), ("w", c_void_p), ("bias", c_void_p), ("bias2", c_void_p), ("res", c_void_p),
                ("y", c_void_p),
                ("B", c_int64), ("Ci", c_int64), ("Co", c_int64), ("Lin", c_int64), ("Lout", c_int64),
                ("ncols", c_int64), ("x_bstride", c_int64), ("y_bstride", c_int64), ("res_bstride", c_int64),
                ("w_bstride", c_int64),
                ("K", c_int), ("stride", c_int), ("dil", c_int), ("pad", c_int), ("groups", c_int),
                ("nphase", c_int), ("ostride", c_int), ("ooffset", c_int),
                ("in_act", c_int), ("out_act", c_int), ("accumulate", c_int), ("_pad0", c_int),
                ("in_scale", c_float), ("in_slope", c_float), ("out_slope", c_float), ("out_scale", c_float),
                ("ntoff", c_int), ("wrap", c_int), ("toff", c_int * 16),
                ("wx", c_void_p), ("wx_nmf", c_int), ("wx_passes", c_int),
                ("amax_in", c_void_p), ("amax_out", c_void_p),
                ("src_x", c_void_p), ("src_w", c_void_p), ("src_b", c_void_p),
                ("src_K", c_int), ("src_stride", c_int), ("src_pad", c_int), ("_pad1", c_int),
                ("src_len", c_int64), ("src_bstride", c_int64)]


class Conv64Args(ctypes.Structure):
    """rvc_conv64_args: the f64 implicit-GEMM conv of the f64 RMVPE (rmvpe64.hip)."""
    _fields_ = [("x", c_void_p), ("w", c_void_p), ("bias", c_void_p), ("res", c_void_p), ("y", c_void_p),
                ("B", c_int64), ("Ci", c_int64), ("Co", c_int64), ("Lin", c_int64), ("Lout", c_int64),
                ("x_bstride", c_int64), ("y_bstride", c_int64), ("res_bstride", c_int64),
                ("K", c_int), ("pad", c_int), ("out_act", c_int), ("y_f32", c_int), ("out_slope", c_double),
                ("ntoff", c_int), ("wrap", c_int), ("toff", c_int * 16),
                ("w_bstride", c_int64), ("w_bmod", c_int), ("_pad0", c_int)]


class Wino64Args(ctypes.Structure):
    """rvc_wino64_args: the f64 Winograd F(4x4, 3x3) conv of RMVPE's deep levels (rmvpe64.hip)."""
    _fields_ = [("x", c_void_p), ("v", c_void_p), ("bias", c_void_p), ("res", c_void_p), ("y", c_void_p),
                ("B", c_int64), ("Ci", c_int64), ("Co", c_int64), ("H", c_int64), ("W", c_int64),
                ("x_bstride", c_int64), ("y_bstride", c_int64), ("res_bstride", c_int64),
                ("out_act", c_int), ("y_f32", c_int)]


class AttnArgs(ctypes.Structure):
    _fields_ = [("q", c_void_p), ("k", c_void_p), ("v", c_void_p), ("o", c_void_p), ("rk", c_void_p),
                ("ev", c_void_p), ("ml", c_void_p),
                ("B", c_int64), ("H", c_int64), ("D", c_int64), ("T", c_int64), ("ldc", c_int64),
                ("q_hs", c_int64), ("k_hs", c_int64), ("v_hs", c_int64), ("o_hs", c_int64),
                ("q_bs", c_int64), ("k_bs", c_int64), ("v_bs", c_int64), ("o_bs", c_int64),
                ("W", c_int), ("_pad0", c_int), ("scale", c_float), ("_pad1", c_float)]


class F0Post(ctypes.Structure):
    """rvc_f0_post: autotune / f0-file steps of VC.get_f0 (convert.py:311-318)."""
    _fields_ = [("autotune", c_int), ("_pad0", c_int), ("strength", c_double), ("rep", c_void_p),
                ("rep_off", c_int64), ("rep_len", c_int64)]


class ResblockArgs(ctypes.Structure):
    """rvc_resblock_args: one fused (convs1[i], convs2[i]) ResBlock pair (residuals.py:22-44)."""
    _fields_ = [("x", c_void_p), ("y", c_void_p), ("w1x", c_void_p), ("b1", c_void_p), ("w2x", c_void_p),
                ("b2", c_void_p), ("C", c_int64), ("L", c_int64), ("K", c_int), ("dil", c_int), ("nmf1", c_int),
                ("nmf2", c_int), ("passes", c_int), ("accumulate", c_int), ("slope", c_float), ("B", c_int)]


class DenoiseArgs(ctypes.Structure):
    """rvc_denoise_args: the non-stationary spectral gate (main/tools/noisereduce.py:124-199)."""
    _fields_ = [("chunk_size", c_int64), ("padding", c_int64), ("n_fft", c_int), ("hop", c_int),
                ("n_movemean", c_int), ("filt_h", c_int), ("filt_w", c_int), ("_pad0", c_int),
                ("prop_decrease", c_double), ("n_thresh", c_double), ("temp_coeff", c_double),
                ("window", c_void_p), ("filt", c_void_p)]


class Param(ctypes.Structure):
    """rvc_param: one named host array of a checkpoint's weight dict (model-level API)."""
    _fields_ = [("name", ctypes.c_char_p), ("data", c_void_p), ("dtype", c_int), ("ndim", c_int),
                ("shape", c_int64 * 4)]


class SynthCfg(ctypes.Structure):
    """rvc_synth_cfg: the .pth "config" list (train.py:729-742)."""
    _fields_ = [("inter_channels", c_int), ("hidden_channels", c_int), ("filter_channels", c_int), ("n_heads", c_int),
                ("n_layers", c_int), ("kernel_size", c_int), ("n_resblocks", c_int), ("n_dilations", c_int),
                ("resblock_kernel_sizes", c_int * 4), ("resblock_dilation_sizes", (c_int * 4) * 4),
                ("n_upsamples", c_int), ("upsample_rates", c_int * 8), ("upsample_kernel_sizes", c_int * 8),
                ("upsample_initial_channel", c_int), ("spk_embed_dim", c_int), ("gin_channels", c_int), ("sr", c_int)]


class ContentVecCfg(ctypes.Structure):
    """rvc_contentvec_cfg: the fairseq .pt cfg["model"] fields the encoder needs (fairseq.py:30-36)."""
    _fields_ = [("encoder_embed_dim", c_int), ("encoder_attention_heads", c_int), ("conv_pos_groups", c_int),
                ("_pad0", c_int)]


class VcArgs(ctypes.Structure):
    """rvc_vc_args: one VC.pipeline segment (convert.py:388-458)."""
    _fields_ = [("sid", c_int64), ("pitch_shift", c_double), ("protect", c_float), ("version", c_int),
                ("x_pad", c_int), ("x_max", c_int), ("tgt_sr", c_int), ("_pad0", c_int), ("index_rate", c_double), ("seed", c_uint64)]


class VcOpts(ctypes.Structure):
    """rvc_vc_opts: VC.pipeline's options beyond one RMVPE segment (f0 method, autotune, f0 file, volume envelope)."""
    _fields_ = [("f0_method", c_int), ("f0_autotune", c_int), ("f0_autotune_strength", c_double),
                ("f0_file", c_void_p), ("f0_file_rows", c_int64), ("volume_envelope", c_double),
                ("crepe_dither", c_void_p)]


class IvfIndex(ctypes.Structure):
    """rvc_ivf_index: a faiss IndexIVFFlat's arrays on the host (rvc_load_index)."""
    _fields_ = [("d", c_int64), ("nlist", c_int64), ("ntotal", c_int64), ("nprobe", c_int), ("_pad0", c_int),
                ("centroids", c_void_p), ("list_off", c_void_p), ("codes", c_void_p), ("ids", c_void_p),
                ("big", c_void_p)]


# name -> argtypes (restype is int unless listed in _RESTYPES)
SIGNATURES = {
    "rvc_last_error": [],
    "rvc_version": [],
    "rvc_conv1d": [POINTER(Conv1dArgs), c_void_p, c_int64, c_void_p],
    "rvc_conv1d_workspace_bytes": [POINTER(Conv1dArgs)],
    "rvc_conv1d_set_probe_event": [c_void_p],
    "rvc_conv1d_set_stamps": [c_void_p, c_int64],
    "rvc_resblock_set_stamps": [c_void_p, c_int64],
    "rvc_resblock_set_ylds": [c_int],
    "rvc_resblock_set_wide64": [c_int],
    "rvc_conv1d_set_tile_epi": [c_int],
    "rvc_conv1d_set_swz": [c_int],
    "rvc_conv1d_set_f16_fast": [c_int],
    "rvc_bigru64_set_f32": [c_int],
    "rvc_conv1d_set_splitk_target": [c_int],
    "rvc_stream_create_cu_mask": [c_void_p, c_int, POINTER(c_void_p)],
    "rvc_stream_destroy": [c_void_p],
    "rvc_conv1d_engine": [POINTER(Conv1dArgs)],
    "rvc_conv1d_x6_bytes": [c_int64, c_int64, c_int, c_int64],
    "rvc_conv1d_pack_x6": [c_void_p, c_int64, c_int64, c_int, c_int64, c_void_p, POINTER(c_int), c_void_p],
    "rvc_conv1d_f16_bytes": [c_int64, c_int64, c_int, c_int64],
    "rvc_pm_frames": [c_int64],
    "rvc_pm_work_bytes": [c_int64],
    "rvc_pm_f0": [c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p],
    "rvc_pm_post": [c_void_p, c_int64, c_int64, ctypes.c_double, c_void_p, c_void_p, c_void_p, c_void_p],
    "rvc_conv1d_pack_f16": [c_void_p, c_int64, c_int64, c_int, c_int64, c_void_p, POINTER(c_int), c_void_p],
    "rvc_attention_workspace_bytes": [POINTER(AttnArgs)],
    "rvc_attention": [POINTER(AttnArgs), c_void_p, c_int64, c_void_p],
    "rvc_attention_amax": [POINTER(AttnArgs), c_void_p, c_void_p, c_int64, c_void_p],
    "rvc_attention_ex": [POINTER(AttnArgs), c_void_p, c_void_p, c_void_p, c_int64, c_void_p],
    "rvc_attention_set_f16": [c_int],
    "rvc_layernorm_cf_amax": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int64, c_float,
                              c_void_p, c_void_p],
    "rvc_textenc_embed": [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int64, c_float, c_float,
                          c_void_p],
    "rvc_textenc_embed_amax": [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int64, c_float, c_float,
                               c_void_p, c_void_p],
    "rvc_layernorm_cf": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int64, c_float,
                         c_void_p],
    "rvc_chnorm_gelu": [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int64, c_float, c_int, c_void_p],
    "rvc_fe0_ws_bytes": [c_int64, c_int64, c_int64],
    "rvc_fe0_gn_gelu": [c_void_p, c_int64, c_int64, c_int64, c_void_p, c_int64, c_int, c_int, c_void_p, c_void_p, c_void_p,
                        c_float, c_int, c_void_p, c_int64, c_void_p],
    "rvc_fe0_gn_gelu_amax": [c_void_p, c_int64, c_int64, c_int64, c_void_p, c_int64, c_int, c_int, c_void_p, c_void_p,
                             c_void_p, c_float, c_int, c_void_p, c_void_p, c_int64, c_void_p],
    "rvc_prior_sample": [c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int64, c_float, c_void_p],
    "rvc_gate": [c_void_p, c_void_p, c_int64, c_int64, c_int64, c_void_p],
    "rvc_flip_channels": [c_void_p, c_void_p, c_int64, c_int64, c_int64, c_void_p],
    "rvc_transpose": [c_void_p, c_void_p, c_int64, c_int64, c_int64, c_void_p],
    "rvc_randn": [c_void_p, c_int64, c_uint64, c_uint64, c_void_p],
    "rvc_randn_ex": [c_void_p, c_int64, c_uint64, c_uint64, c_void_p, c_void_p],
    "rvc_rand_triang": [c_void_p, c_int64, c_float, c_float, c_uint64, c_uint64, c_void_p, c_void_p],
    "rvc_sine_source": [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int, c_float, c_float, c_float,
                        c_void_p],
    "rvc_stft_frames": [c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int, c_int, c_void_p],
    "rvc_spec_mag": [c_void_p, c_void_p, c_int64, c_int64, c_void_p],
    "rvc_stft_mag": [c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int64, c_int, c_int, c_int64, c_int64, c_void_p],
    "rvc_mel_image": [c_void_p, c_void_p, c_int64, c_int64, c_int64, c_float, c_float, c_void_p],
    "rvc_avgpool2": [c_void_p, c_void_p, c_int64, c_int64, c_int64, c_void_p],
    "rvc_interleave4": [c_void_p, c_void_p, c_int64, c_int64, c_int64, c_void_p],
    "rvc_img_to_seq": [c_void_p, c_void_p, c_int64, c_int64, c_int64, c_void_p],
    "rvc_bigru": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p],
    "rvc_bigru_set_spin_limit": [ctypes.c_uint],
    "rvc_bigru_batched": [c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_int64, c_int64,
                          c_void_p],
    "rvc_conv64": [POINTER(Conv64Args), c_void_p, c_int64, c_void_p],
    "rvc_conv64_workspace_bytes": [POINTER(Conv64Args)],
    "rvc_conv64_plan": [POINTER(Conv64Args), POINTER(c_int)],
    "rvc_wino64_use": [c_int64, c_int64, c_int64, c_int64],
    "rvc_wino64_weights": [c_void_p, c_void_p, c_int64, c_int64, c_void_p],
    "rvc_wino64_workspace_bytes": [POINTER(Wino64Args)],
    "rvc_wino64_conv": [POINTER(Wino64Args), c_void_p, c_int64, c_void_p],
    "rvc_conv64_set_plan": [c_int, c_int, c_int],
    "rvc_stft_mag64": [c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int64, c_int, c_int, c_int64, c_int64,
                       c_void_p],
    "rvc_mel_image64": [c_void_p, c_void_p, c_int64, c_int64, c_int64, c_int64, c_double, c_double, c_int64, c_int64,
                        c_void_p],
    "rvc_avgpool2_64": [c_void_p, c_void_p, c_int64, c_int64, c_int64, c_int64, c_int64, c_int64, c_void_p],
    "rvc_interleave4_64": [c_void_p, c_void_p, c_int64, c_int64, c_int64, c_int64, c_int64, c_int64, c_void_p],
    "rvc_img_to_seq64": [c_void_p, c_void_p, c_int64, c_int64, c_int64, c_int64, c_int64, c_int64, c_void_p],
    "rvc_bigru64_batched": [c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_int64,
                            c_int64, c_void_p],
    "rvc_rmvpe_decode": [c_void_p, c_int64, c_int64, c_double, c_double, POINTER(F0Post), c_void_p, c_void_p,
                         c_void_p, c_void_p],
    "rvc_filtfilt_work_bytes": [c_int64],
    "rvc_filtfilt_pad": [c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p,
                         c_void_p],
    "rvc_ivf_coarse_ws_bytes": [c_int64, c_int64],
    "rvc_ivf_search": [c_void_p, c_int64, c_int64, c_int64, c_int64, c_void_p, c_int64, c_int, c_void_p, c_void_p,
                       c_void_p, c_int, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p],
    "rvc_ivf_search_ex": [c_void_p, c_int64, c_int64, c_int64, c_int64, c_void_p, c_int64, c_int, c_void_p, c_void_p,
                       c_void_p, c_int, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_int, c_void_p],
    "rvc_ivf_blend": [c_void_p, c_int64, c_int64, c_int64, c_int64, c_void_p, c_void_p, c_int, c_void_p, c_int64,
                      c_double, c_void_p, c_int64, c_int64, c_void_p],
    "rvc_crepe_frames": [c_void_p, c_int64, c_int, c_int64, c_int64, c_void_p, c_void_p],
    "rvc_bn_maxpool": [c_void_p, c_int64, c_int64, c_int64, c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int64,
                       c_void_p],
    "rvc_crepe_decode_ws_bytes": [c_int64],
    "rvc_crepe_decode": [c_void_p, c_int64, c_int, c_int, c_void_p, c_int, c_void_p, c_double, c_double, c_void_p,
                         c_void_p, c_int64, c_void_p, c_void_p, c_void_p],
    "rvc_crepe_smooth_coarse": [c_void_p, c_void_p, c_int64, c_float, c_double, c_double, POINTER(F0Post), c_void_p,
                                c_void_p, c_void_p],
    "rvc_phone_upsample": [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int64, c_float, c_void_p],
    "rvc_peak_normalize": [c_void_p, c_int64, c_void_p, c_void_p, c_void_p],
    "rvc_rms_frames_len": [c_int64, c_int64],
    "rvc_rms_frames": [c_void_p, c_void_p, c_int64, c_int64, c_void_p, c_void_p],
    "rvc_rms_mix": [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_double, c_void_p],
    "rvc_denoise_work_bytes": [c_int64, POINTER(DenoiseArgs)],
    "rvc_resblock_lds_bytes": [c_int64, c_int, c_int, c_int],
    "rvc_resblock_pair": [POINTER(ResblockArgs), c_void_p],
    "rvc_denoise": [c_void_p, c_int64, POINTER(DenoiseArgs), c_void_p, c_int64, c_void_p, c_void_p],
    "rvc_ctx_create": [c_int, POINTER(c_void_p)],
    "rvc_ctx_destroy": [c_void_p],
    "rvc_ctx_set_precision": [c_void_p, c_int],
    "rvc_ctx_set_rmvpe_precision": [c_void_p, c_int],
    "rvc_load_synth": [c_void_p, POINTER(Param), c_int, POINTER(SynthCfg)],
    "rvc_synth_out_len": [c_void_p, c_int64],
    "rvc_load_contentvec": [c_void_p, POINTER(Param), c_int, POINTER(ContentVecCfg)],
    "rvc_contentvec_frames": [c_int64],
    "rvc_contentvec_forward": [c_void_p, c_void_p, c_int64, c_int64, c_int, c_int, c_void_p, c_void_p],
    "rvc_load_rmvpe": [c_void_p, POINTER(Param), c_int],
    "rvc_rmvpe_frames": [c_int64],
    "rvc_rmvpe_salience_ld": [c_int64],
    "rvc_rmvpe_forward": [c_void_p, c_void_p, c_int64, c_int64, c_void_p, c_void_p],
    "rvc_rmvpe_check": [c_void_p],
    "rvc_load_crepe": [c_void_p, POINTER(Param), c_int],
    "rvc_vc_out_len": [c_void_p, c_int64, POINTER(VcArgs)],
    "rvc_load_index": [c_void_p, POINTER(IvfIndex)],
    "rvc_device_bytes_in_use": [],
    "rvc_pm_windows": [c_void_p, c_void_p],
    "rvc_f0_file_resample": [c_void_p, c_int64, c_void_p, c_int64],
    "rvc_quiet_points_count": [c_int64, c_int, c_int64, c_int64],
    "rvc_quiet_points_ws_bytes": [c_int64, c_int, c_int64, c_int64, c_int64],
    "rvc_quiet_points": [c_void_p, c_int64, c_int, c_int64, c_int64, c_int64, c_void_p, c_int64, c_void_p, c_void_p],
    "rvc_vc_convert": [c_void_p, c_void_p, c_int64, POINTER(VcArgs), c_void_p, c_void_p],
    "rvc_vc_convert_ex": [c_void_p, c_void_p, c_int64, POINTER(VcArgs), c_void_p, c_void_p, c_int64,
                          POINTER(c_int64), c_void_p],
    "rvc_crepe_f0": [c_void_p, c_void_p, c_int64, c_void_p, c_uint64, c_double, c_void_p, c_void_p, c_void_p,
                     c_void_p, c_void_p],
    "rvc_synth_infer": [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_void_p, c_void_p, c_void_p, c_uint64,
                        c_void_p, c_void_p],
}
_RESTYPES = {"rvc_last_error": ctypes.c_char_p, "rvc_conv1d_workspace_bytes": c_int64, "rvc_conv1d_x6_bytes": c_int64,
             "rvc_conv64_workspace_bytes": c_int64, "rvc_wino64_workspace_bytes": c_int64,
             "rvc_conv1d_f16_bytes": c_int64, "rvc_pm_frames": c_int64, "rvc_pm_work_bytes": c_int64,
             "rvc_filtfilt_work_bytes": c_int64, "rvc_attention_workspace_bytes": c_int64,
             "rvc_ivf_coarse_ws_bytes": c_int64, "rvc_crepe_decode_ws_bytes": c_int64,
             "rvc_rms_frames_len": c_int64, "rvc_denoise_work_bytes": c_int64, "rvc_resblock_lds_bytes": c_int64, "rvc_bigru_set_spin_limit": ctypes.c_uint,
             "rvc_ctx_destroy": None, "rvc_conv1d_set_probe_event": None, "rvc_synth_out_len": c_int64,
             "rvc_contentvec_frames": c_int64, "rvc_rmvpe_frames": c_int64, "rvc_rmvpe_salience_ld": c_int64,
             "rvc_vc_out_len": c_int64, "rvc_device_bytes_in_use": c_int64,
             "rvc_quiet_points_count": c_int64, "rvc_f0_file_resample": c_int64, "rvc_quiet_points_ws_bytes": c_int64,
             "rvc_fe0_ws_bytes": c_int64}

_lib = None


def load():
    """Load the HIP library once; raise loudly if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"rvc_amd: HIP library not built ({LIB_PATH}); run __graft_entry__.build() "
                           "or `make -C rvc-maker_amd/csrc`. There is no CPU fallback.")
    lib = ctypes.CDLL(LIB_PATH)
    for name, argt in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = argt
        fn.restype = _RESTYPES.get(name, c_int)
    _lib = lib
    return lib


def check(rc: int, what: str):
    if rc != 0:
        raise RuntimeError(f"rvc_amd: {what} failed ({rc}): {load().rvc_last_error().decode()}")
