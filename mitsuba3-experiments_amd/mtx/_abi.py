"""ctypes mirror of include/mtx.h (plain C structs, no torch types)."""
from __future__ import annotations

import ctypes as C

MTX_ABI_VERSION = 8

MTX_MAT_DIFFUSE = 1
MTX_MAT_ROUGHPLASTIC = 2
MTX_MAT_CONDUCTOR = 3
MTX_MAT_ROUGHCONDUCTOR = 4
MTX_MAT_DIELECTRIC = 5
MTX_MAT_ROUGHDIELECTRIC = 6

MTX_MF_TWOSIDED = 1
MTX_MF_MASK = 2
MTX_MF_BECKMANN = 4
MTX_MF_NONLINEAR = 8

MTX_INT_PATH = 1
MTX_INT_PATH_MIS = 2
MTX_INT_NRC = 3
MTX_INT_PSSMLT_SIMPLE = 4
MTX_INT_RESTIR_GI = 5
MTX_INT_PSSMLT_PATH = 6
MTX_INT_NERAD_RHS = 7
MTX_INT_NERAD = 8
MTX_INT_SIMPLE = 9

MTX_RESTIR_BIAS_CORRECTION = 1
MTX_RESTIR_JACOBIAN = 2
MTX_RESTIR_BSDF_SAMPLING = 4
MTX_RESTIR_SPATIAL_SPATIAL = 8
MTX_RESTIR_STAGE_A = 16
MTX_RENDER_STATS = 1
MTX_RENDER_TIMING = 2
MTX_RENDER_NRC_CACHE = 4
MTX_RESTIR_STAGE_B = 32

MTX_ROUGH_TRANSMITTANCE_RES = 64
MTX_BVH_WIDTH = 4          # closest-hit BVH (mtx.h)
MTX_BVH_MAX_LEAF = 8
MTX_BVH_NODE_WORDS = 16
MTX_BVH_MAX_DEPTH = 40
MTX_OCC_WIDTH = 8          # occlusion (any-hit) BVH
MTX_OCC_MAX_LEAF = 3
MTX_OCC_NODE_WORDS = 20

ERRORS = {-1: "MTX_E_ARG", -2: "MTX_E_HIP", -3: "MTX_E_NOSCENE", -4: "MTX_E_OOM", -5: "MTX_E_UNSUPPORTED"}


class Material(C.Structure):
    _fields_ = [
        ("type", C.c_uint32),
        ("flags", C.c_uint32),
        ("tex", C.c_int32),
        ("opacity", C.c_float),
        ("rgb", C.c_float * 3),
        ("alpha", C.c_float),
        ("eta", C.c_float),
        ("eta_rgb", C.c_float * 3),
        ("k_rgb", C.c_float * 3),
        ("spec_weight", C.c_float),
        ("internal_refl", C.c_float),
        ("table", C.c_int32),
    ]


class Texture(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("offset", C.c_uint64)]


class Emitter(C.Structure):
    _fields_ = [
        ("center", C.c_float * 3),
        ("col0", C.c_float * 3),
        ("col1", C.c_float * 3),
        ("normal", C.c_float * 3),
        ("inv_area", C.c_float),
        ("radiance", C.c_float * 3),
    ]


class Shape(C.Structure):
    _fields_ = [("material", C.c_uint32), ("emitter", C.c_int32), ("flags", C.c_uint32), ("pad", C.c_uint32)]


class Camera(C.Structure):
    _fields_ = [
        ("origin", C.c_float * 3),
        ("axis_x", C.c_float * 3),
        ("axis_y", C.c_float * 3),
        ("axis_z", C.c_float * 3),
        ("tan_x", C.c_float),
        ("tan_y", C.c_float),
        ("near_clip", C.c_float),
        ("far_clip", C.c_float),
        ("width", C.c_uint32),
        ("height", C.c_uint32),
        ("inv_rows", C.c_float * 9),
        ("pad", C.c_uint32),
    ]


class SceneDesc(C.Structure):
    _fields_ = [
        ("n_tris", C.c_uint32),
        ("n_nodes", C.c_uint32),
        ("n_verts", C.c_uint32),
        ("n_shapes", C.c_uint32),
        ("n_materials", C.c_uint32),
        ("n_emitters", C.c_uint32),
        ("n_textures", C.c_uint32),
        ("flags", C.c_uint32),
        ("nodes", C.c_void_p),
        ("tri_geom", C.c_void_p),
        ("tri_vidx", C.c_void_p),
        ("tri_shape", C.c_void_p),
        ("vpos", C.c_void_p),
        ("vnormal", C.c_void_p),
        ("vuv", C.c_void_p),
        ("shapes", C.c_void_p),
        ("materials", C.c_void_p),
        ("emitters", C.c_void_p),
        ("textures", C.c_void_p),
        ("texels", C.c_void_p),
        ("n_texels", C.c_uint64),
        ("tables", C.c_void_p),
        ("n_tables", C.c_uint32),
        ("pad0", C.c_uint32),
        ("camera", Camera),
        ("occ_nodes", C.c_void_p),
        ("occ_tri_geom", C.c_void_p),
        ("n_occ_nodes", C.c_uint32),
        ("pad1", C.c_uint32),
        ("occ_perm", C.c_void_p),
        ("env_radiance", C.c_float * 3),
        ("has_env", C.c_uint32),
    ]


class RenderArgs(C.Structure):
    _fields_ = [
        ("integrator", C.c_uint32),
        ("max_depth", C.c_uint32),
        ("rr_depth", C.c_uint32),
        ("seed", C.c_uint32),
        ("spp", C.c_uint32),
        ("spp_total", C.c_uint32),
        ("sample_offset", C.c_uint32),
        ("y0", C.c_uint32),
        ("y1", C.c_uint32),
        ("chunk_paths", C.c_uint32),
        ("nrc_c", C.c_float),
        ("flags", C.c_uint32),
        ("iterations", C.c_uint32),
        ("frame", C.c_uint32),
        ("restir_flags", C.c_uint32),
        ("max_M_temporal", C.c_uint32),
        ("max_M_spatial", C.c_uint32),
        ("initial_search_radius", C.c_float),
        ("minimal_search_radius", C.c_float),
        ("reserved", C.c_uint32),
    ]


class FieldDesc(C.Structure):
    _fields_ = [
        ("n_levels", C.c_uint32),
        ("n_features", C.c_uint32),
        ("log2_table", C.c_uint32),
        ("base_res", C.c_uint32),
        ("per_level_scale", C.c_float),
        ("bbox_min", C.c_float * 3),
        ("bbox_max", C.c_float * 3),
        ("n_in", C.c_uint32),
        ("n_hidden", C.c_uint32),
        ("table", C.c_void_p),
        ("weights", C.c_void_p),
    ]


class Stats(C.Structure):
    _fields_ = [
        ("rays_closest", C.c_uint64),
        ("rays_shadow", C.c_uint64),
        ("nodes_closest", C.c_uint64),
        ("tris_closest", C.c_uint64),
        ("nodes_shadow", C.c_uint64),
        ("tris_shadow", C.c_uint64),
        ("trace_launches", C.c_uint64),
        ("shadow_launches", C.c_uint64),
        ("trace_ms", C.c_double),
        ("shadow_ms", C.c_double),
        ("shade_ms", C.c_double),
        ("other_ms", C.c_double),
        ("paths", C.c_uint64),
        ("wave_node_iters", C.c_uint64),
        ("wave_leaf_iters", C.c_uint64),
        ("cache_queries", C.c_uint64),
        ("cache_encode_ms", C.c_double),
        ("cache_mlp_ms", C.c_double),
        ("streams", C.c_uint32),
        ("reserved", C.c_uint32),
    ]

    def as_dict(self) -> dict:
        return {name: getattr(self, name) for name, _ in self._fields_}


class FieldOpt(C.Structure):
    _fields_ = [
        ("lr", C.c_float),
        ("beta_1", C.c_float),
        ("beta_2", C.c_float),
        ("epsilon", C.c_float),
        ("init_scale", C.c_float),
        ("growth_factor", C.c_float),
        ("backoff_factor", C.c_float),
        ("growth_interval", C.c_uint32),
    ]


class TrainStats(C.Structure):
    _fields_ = [
        ("loss", C.c_double),
        ("scale", C.c_float),
        ("found_inf", C.c_uint32),
        ("step", C.c_uint32),
        ("rhs_queries", C.c_uint32),
        ("ms_lhs", C.c_double),
        ("ms_rhs", C.c_double),
        ("ms_train", C.c_double),
        ("ms_total", C.c_double),
        ("ms_trace", C.c_double),
        ("rays_closest", C.c_uint64),
        ("nodes_closest", C.c_uint64),
        ("tris_closest", C.c_uint64),
    ]

    def as_dict(self) -> dict:
        return {name: getattr(self, name) for name, _ in self._fields_}


class NeradTables(C.Structure):
    _fields_ = [
        ("n_shapes", C.c_uint32),
        ("n_entries", C.c_uint32),
        ("shape_pmf", C.c_void_p),
        ("shape_cdf", C.c_void_p),
        ("shape_sum", C.c_float),
        ("shape_norm", C.c_float),
        ("shape_valid", C.c_uint32 * 2),
        ("tri_off", C.c_void_p),
        ("tri_pmf", C.c_void_p),
        ("tri_cdf", C.c_void_p),
        ("tri_prim", C.c_void_p),
        ("tri_sum", C.c_void_p),
        ("tri_norm", C.c_void_p),
        ("tri_valid", C.c_void_p),
    ]


class NeradArgs(C.Structure):
    _fields_ = [("lhs_seed", C.c_uint32), ("rhs_seed", C.c_uint32), ("batch", C.c_uint32), ("M", C.c_uint32),
                ("flags", C.c_uint32)]


# Every symbol include/mtx.h declares (checked by tests/test_abi.py).
EXPORTS = [
    "mtx_abi_version",
    "mtx_last_error",
    "mtx_ctx_create",
    "mtx_ctx_destroy",
    "mtx_bvh_build",
    "mtx_bvh_build_occlusion",
    "mtx_roughplastic_tables",
    "mtx_scene_upload",
    "mtx_render",
    "mtx_set_camera",
    "mtx_restir_rows",
    "mtx_restir_state",
    "mtx_sample_rays",
    "mtx_sample_rays_dev",
    "mtx_trace",
    "mtx_trace_dev",
    "mtx_prefix_sum_u32",
    "mtx_prefix_sum_f32_hs",
    "mtx_prefix_sum_u32_dev",
    "mtx_prefix_sum_f32_hs_dev",
    "mtx_hashgrid_build",
    "mtx_hashgrid_build_dev",
    "mtx_scatter_reduce_f32",
    "mtx_scatter_reduce_f32_dev",
    "mtx_group_by_u32",
    "mtx_group_by_u32_dev",
    "mtx_field_upload",
    "mtx_field_features",
    "mtx_field_mlp",
    "mtx_field_eval",
    "mtx_last_device_ms",
    "mtx_field_train_init",
    "mtx_field_grad",
    "mtx_field_train_step",
    "mtx_field_params",
    "mtx_nerad_upload",
    "mtx_nerad_lhs",
    "mtx_nerad_rhs",
    "mtx_nerad_step",
]
