from .modules import Int8Params, Linear4bit, Linear8bitLt, LinearFP4, LinearNF4, Params4bit  # noqa: F401
