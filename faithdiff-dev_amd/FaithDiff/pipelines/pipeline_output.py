"""Mirror of FaithDiff/pipelines/pipeline_output.py:11-21."""
from dataclasses import dataclass
from typing import List, Union

import numpy as np
import PIL.Image


@dataclass
class FaithDiffStableDiffusionXLPipelineOutput:
    """images: list of PIL images or an (N, H, W, 3) numpy array."""
    images: Union[List[PIL.Image.Image], np.ndarray]

    def __getitem__(self, i):  # diffusers BaseOutput tuple-style access
        return (self.images,)[i]
