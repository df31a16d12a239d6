from ._functions import MatmulLtState, MatMul4Bit, MatMul8bitLt, matmul, matmul_4bit  # noqa: F401
