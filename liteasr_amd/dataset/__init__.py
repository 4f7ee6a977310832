from .asr_dataset import AudioFileDataset  # noqa: F401
from .liteasr_dataset import LiteasrDataset  # noqa: F401
