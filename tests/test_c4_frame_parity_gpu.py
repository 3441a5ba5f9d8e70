"""C4 (final_scene 800x800, 4900 spp, depth 40) against the f64 oracle on the rows that
test_baseline_config_frames_vs_oracle does not compare (rows 0, 1 and 3 mod 4: 600 rows, 2.35 G
samples), so that together with its five bands the WHOLE frame is compared (DESIGN
§8.1). Same checks as those bands: product, counting and interpreter kernels bit-identical, per
pixel within TOL of the oracle with identical NaN / inf masks, op counts within C4_OPS_RTOL.

About four minutes of oracle time per 200-row band on the box's 16 host threads, so opt-in
(RT_FULL_FRAME_PARITY=1) rather than part of the default -m gpu run."""
import os

import pytest

import surely_rt as rt
from test_gpu_parity import C4_OPS_RTOL, _compare, _frame_report

pytestmark = [
    pytest.mark.gpu,
    pytest.mark.skipif(os.environ.get("RT_FULL_FRAME_PARITY") != "1",
                       reason="whole-frame C4 parity is opt-in: RT_FULL_FRAME_PARITY=1"),
]


@pytest.mark.timeout(900)
@pytest.mark.parametrize("b", [0, 1, 3])
def test_c4_remaining_rows_vs_oracle(gpu_available, b):
    blob, cam = rt.preset_blob("final_scene", width=800, spp=5000, depth=40)
    acc_g, acc_o, st = _compare(blob, cam, row_begin=b, row_step=4, n_rows=200,
                                ops_rtol=C4_OPS_RTOL)
    assert st.samples == 200 * 800 * cam.samples_per_pixel
    _frame_report(f"C4 rows {b} mod 4", acc_g, acc_o, cam.samples_per_pixel)
