"""The CPU-path parity tests (test_cpu_path.py: the product's host-core cdequantize_blockwise_cpu_fp32 /
cquantize_blockwise_cpu_fp32, ref:sycl/cpu_ops.cpp:7-63 + ref:sycl/common.cpp:4-35, bit-exact against the golden
fixtures, the oracle and the reference-shaped port) collected a second time under the `gpu` mark, so the driver's
`pytest -m gpu` run on the GPU box checks them on that box's host cores too.  They need no GPU; the CPU suite
(`-m "not gpu"`) runs the originals."""
import pytest

from test_cpu_path import (test_config1_nf4_bytes_dequant_matches_port, test_cpu_path_golden,  # noqa: F401
                           test_cpu_path_vs_oracle_and_port, test_functional_cpu_route)

pytestmark = pytest.mark.gpu
