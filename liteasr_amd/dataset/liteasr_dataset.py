"""Dataset interface (liteasr/dataset/liteasr_dataset.py:15-32)."""

from torch.utils.data import Dataset


class LiteasrDataset(Dataset):
    def batchify(self, dataset_cfg) -> None:
        raise NotImplementedError

    def set_postprocess(self, postprocess_cfg) -> None:
        raise NotImplementedError

    def collator(self, samples):
        raise NotImplementedError

    def __getitem__(self, index: int):
        raise NotImplementedError

    def __len__(self) -> int:
        raise NotImplementedError
