"""Documentation citations of the C header stay in step with it (stale line
numbers in INTEGRATION.md)."""
import re
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent


def test_integration_header_citations_point_at_their_structs():
    header = (REPO / "include" / "rt_mi355x.h").read_text().splitlines()
    text = (REPO / "INTEGRATION.md").read_text()
    cites = re.findall(r"pub struct (\w+) \{\s*// rt_mi355x\.h:(\d+)-(\d+)", text)
    assert len(cites) >= 4
    names = {"RtSceneBlob": "rt_scene_blob", "RtCamera": "rt_camera",
             "RtRenderOpts": "rt_render_opts", "RtStats": "rt_stats"}
    for rust, a, b in cites:
        a, b = int(a), int(b)
        assert header[a - 1].startswith(f"typedef struct {names[rust]}"), (rust, a)
        assert header[b - 1].startswith(f"}} {names[rust]};"), (rust, b)
    for m in re.finditer(r"rt_mi355x\.h:(\d+)-(\d+)\)", text):  # flag block citation
        a, b = int(m.group(1)), int(m.group(2))
        assert "RT_FLAG_" in header[a - 1] and "RT_FLAG_" in "\n".join(header[a - 1:b])
