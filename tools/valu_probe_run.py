"""Runs tools/valu_probe (built in-tree beforehand: hipcc --offload-arch=gfx950 -O3 tools/valu_probe.hip
-o tools/valu_probe) as a child process and prints its table."""
import os
import subprocess
import sys

exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "valu_probe")
sys.exit(subprocess.call([exe]))
