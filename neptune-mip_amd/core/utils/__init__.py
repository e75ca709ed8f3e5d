from .data import Data
from .input_to_data import check_input, data_to_solver_input
