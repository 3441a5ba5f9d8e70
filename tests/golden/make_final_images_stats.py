"""Generate tests/golden/final_images_stats.json from the reference's own renders.

The reference (Rust, unseeded, no tests) ships its only outputs as PNGs under
/root/reference/final_images/. They cannot be reproduced bit-for-bit (unseeded RNG, SURVEY
§0.2), so parity is pinned statistically: mean sRGB8, the exact count of pure-black pixels (a
geometric property of the Cornell camera), and block means on a grid.

Run here (the reference is not present on the GPU box):  python tests/golden/make_final_images_stats.py
"""
import json
from pathlib import Path

import numpy as np
from PIL import Image

SRC = Path("/root/reference/final_images")
OUT = Path(__file__).resolve().parent / "final_images_stats.json"

# which scene/config produced each image
META = {
    "book3.png": {"preset": "cornell_box", "variant": "", "width": 600, "spp": 1000, "depth": 50},
    "mixed_pdf.png": {"preset": "cornell_box", "variant": "mixed_pdf", "width": 600, "spp": 1000,
                      "depth": 50},
    "cornell_smoke.png": {"preset": "cornell_smoke", "variant": "", "width": 600, "spp": 100,
                          "depth": 10},
}


def srgb8_to_linear(u8: np.ndarray) -> np.ndarray:
    """Invert color.rs linear_to_gamma at the bin centre of each byte (approximate)."""
    g = (u8.astype(np.float64) + 0.5) / 256.0
    return np.where(g <= 12.92 * 0.0031308, g / 12.92, ((g + 0.055) / 1.055) ** 2.4)


def block_means(a: np.ndarray, grid: int) -> np.ndarray:
    h, w, c = a.shape
    return a.reshape(grid, h // grid, grid, w // grid, c).mean(axis=(1, 3))


def main():
    stats = {}
    for name, meta in META.items():
        img = np.asarray(Image.open(SRC / name).convert("RGB"))
        flat = img.reshape(-1, 3)
        stats[name] = {
            **meta,
            "shape": list(img.shape),
            "mean_srgb8": flat.mean(0).round(4).tolist(),
            "black_pixels": int((flat.sum(1) == 0).sum()),
            "block20_srgb8": block_means(img.astype(np.float64), 20).round(3).tolist(),
            "block10_linear": block_means(srgb8_to_linear(img), 10).round(6).tolist(),
        }
    OUT.write_text(json.dumps(stats, indent=1))
    print(f"wrote {OUT}")


if __name__ == "__main__":
    main()
