from .misc import (  # noqa: F401
    set_seed, text_to_token_ids, token_ids_to_text, read_text_file, read_json_file,
    get_num_params, get_total_size, model_memory_size, start_memory_tracking,
    print_memory_usage, plot_losses, login_hf,
)
from ..config import datasize_mapping, datatype_mapping, model_params_mapping  # noqa: F401
