"""The forward-GEMM routing set read from the TunableOp file (utils/gemm_tuning._tuned_tn): only bf16 TN rows with
the contiguous leading dimensions count."""
from llm_fine_tune_distributed_amd.utils.gemm_tuning import _tuned_tn


def test_tuned_tn_keeps_only_contiguous_bf16_tn_rows(tmp_path):
    p = tmp_path / "t.csv"
    p.write_text(
        "Validator,PT_VERSION,2.10.0\n"
        "GemmTunableOp_BFloat16_TN,tn_3072_8192_2048_ld_2048_2048_3072,Gemm_Rocblas_1,0.04\n"
        "GemmTunableOp_Half_TN,tn_2048_8192_2048_ld_2048_2048_2048,Gemm_Hipblaslt_2,0.03\n"
        "GemmTunableOp_float_TN,tn_4096_8192_2048_ld_2048_2048_4096,Gemm_Hipblaslt_3,0.03\n"
        "GemmTunableOp_BFloat16_NN,nn_2048_8192_3072_ld_2048_3072_2048,Gemm_Rocblas_4,0.05\n"
        "GemmTunableOp_BFloat16_TN,tn_2048_8192_11008_ld_11136_11008_2048,Gemm_Rocblas_5,0.1\n"
        "GemmTunableOp_BFloat16_TN,tn_bad_row\n")
    assert _tuned_tn(str(p)) == frozenset({(3072, 8192, 2048)})


def test_tuned_tn_missing_file_is_empty(tmp_path):
    assert _tuned_tn(str(tmp_path / "none.csv")) == frozenset()


def test_shipped_selections_cover_the_headline_shapes():
    import os
    from llm_fine_tune_distributed_amd.utils import gemm_tuning
    shapes = _tuned_tn(gemm_tuning._DEFAULT)
    assert os.path.exists(gemm_tuning._DEFAULT)
    assert all(len(s) == 3 for s in shapes)
