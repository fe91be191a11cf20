"""JPEG ingest timing alone (bench.py's jpeg_ingest_timing: 8192 reference 720p frames from host
bytes to [B,3,224,224] bf16, fused decode+transform vs the two-step path vs Pillow).
usage: python scripts/jpeg_ingest_micro.py [frames]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    print(json.dumps(bench.jpeg_ingest_timing(torch.device("cuda:0"), 224, B=B)), flush=True)
