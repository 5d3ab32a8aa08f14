from .divrec_logger import get_file_handler, get_logger, get_stream_handler
from .string_utils import to_camel_case

__all__ = ["get_logger", "get_file_handler", "get_stream_handler", "to_camel_case"]
