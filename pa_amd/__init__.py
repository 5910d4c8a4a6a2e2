"""pa_amd: MI355X-native page encode/decode engine for the strawboat format
(drop-in for the codec path of b41sh/pa).  See DESIGN.md."""
from ._native import StrawboatError, build, lib  # noqa: F401
from .read import (  # noqa: F401
    ColumnDecoder,
    ColumnMeta,
    Context,
    NativeReader,
    PageMeta,
    batch_read_array,
    column_iter_to_arrays,
    default_context,
    read_meta,
    unpack_bitmap,
)
from .write import (DeviceColumn, NativeWriter, WriteOptions, assemble_file, encode_column, encode_column_device,  # noqa: F401,E402
                    encode_page, encode_table_device, page_seed)
from .shard import (Shard, exclusive_bases, gather_sizes, rebase_offsets, shard_base, shard_pages,  # noqa: F401,E402
                    shard_slice)
from .binary import (  # noqa: F401,E402
    BINARY, LARGE_BINARY, LARGE_UTF8, UTF8, BinaryColumnDecoder, batch_read_binary, encode_binary_column,
    encode_binary_column_device,
)
from .nested import (DeviceArray, Field, FieldDecoder, HostArray, ListColumnDecoder, NestedColumnDecoder,  # noqa: F401,E402
                     batch_read_field, batch_read_list, encode_field, encode_list_column, encode_list_column_device)
from .file import Leaf, StrawboatFile, parse_schema  # noqa: F401,E402
from .table import ColumnGroupDecoder  # noqa: F401,E402
from .stream import PageArray, decode_columns, iter_page_arrays, to_host  # noqa: F401,E402
