"""Regenerates tests/golden/sampler_golden.npy from libstdc++ (GCC 11, this image's toolchain).

The reference's IncoherentSampler is std::mt19937_64 + std::uniform_real_distribution<float>
(a third-party algorithm: libstdc++'s engine and generate_canonical).  The fixture holds the
first 1000 draws (as float32 bit patterns) for six pixel seeds of main.cpp:73.
"""
import os
import subprocess
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

if __name__ == "__main__":
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "gen")
        subprocess.run(["g++", "-O2", "-std=c++17", os.path.join(HERE, "gen_sampler_golden.cpp"), "-o", exe], check=True)
        txt = subprocess.run([exe], check=True, capture_output=True, text=True).stdout
    arr = np.array([[int(x) for x in line.split()] for line in txt.strip().splitlines()], dtype=np.uint32)
    np.save(os.path.join(HERE, "sampler_golden.npy"), arr)
    print(arr.shape)
