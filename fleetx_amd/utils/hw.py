"""MI355X (gfx950) hardware constants used for MFU / roofline reporting.

Dense (no 2:1 sparsity) matrix-core peaks per GPU; the bench, the train log
line and the layout planner all price against these."""
PEAK_DENSE_FLOPS = {
    "bfloat16": 2.5e15,
    "float16": 2.5e15,
    "float32": 157.3e12,   # vector/MFMA fp32
}
HBM_BYTES_PER_S = 8.0e12
HBM_BYTES = 288 * 2 ** 30


def peak_flops(dtype_name="bfloat16"):
    return PEAK_DENSE_FLOPS.get(str(dtype_name).replace("torch.", ""), PEAK_DENSE_FLOPS["bfloat16"])
