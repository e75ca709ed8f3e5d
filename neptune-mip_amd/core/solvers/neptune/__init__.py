from .neptune import (NeptuneBase, NeptuneMinDelay, NeptuneMinDelayAndUtilization, NeptuneMinUtilization,  # noqa: F401
                      NeptuneWithEFTTCMinDelay, NeptuneWithEFTTCMinDelayAndUtilization, NeptuneWithEFTTCMinUtilization)
from .neptune_step import (NeptuneStep1CPUBase, NeptuneStep1CPUMinDelay,  # noqa: F401
                           NeptuneStep1CPUMinDelayAndUtilization, NeptuneStep1CPUMinUtilization,
                           NeptuneStep2Base, NeptuneStep2MinDelay, NeptuneStep2MinDelayAndUtilization,
                           NeptuneStep2MinUtilization, NeptuneStepBase)
from .output import convert_c_matrix, convert_x_matrix  # noqa: F401
