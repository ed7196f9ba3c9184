"""PipelineVolume: a volume passed between ops that carries its producers as dependencies.

Reference: `sdk/python/kfp/dsl/_pipeline_volume.py:26-104`."""
from __future__ import annotations

from ..k8s import V1PersistentVolumeClaimVolumeSource, V1Volume


class PipelineVolume(V1Volume):
    def __init__(self, pvc=None, volume: V1Volume | None = None, **kwargs):
        if pvc and "name" not in kwargs:
            raise ValueError("Please provide name.")
        if volume and kwargs:
            raise ValueError("You can't pass a volume along with other kwargs.")
        if volume:
            init = {a: getattr(volume, a) for a in self.attribute_map}
        else:
            init = {"name": kwargs.pop("name", None)}
            if pvc and kwargs:
                raise ValueError("You can only pass 'name' along with 'pvc'.")
            if pvc:
                init["persistent_volume_claim"] = V1PersistentVolumeClaimVolumeSource(claim_name=pvc)
        super().__init__(**init, **kwargs)
        self.dependent_names = []

    def after(self, *ops) -> "PipelineVolume":
        """Copy of self depending on `ops`, dropping dependencies already implied by them."""
        from ._pipeline import Pipeline

        def implies(newdep, olddep_name) -> bool:
            if newdep.name == olddep_name:
                return True
            for parent in newdep.dependent_names:
                if parent == olddep_name:
                    return True
                p = Pipeline.get_default_pipeline()
                parent_op = p.ops.get(parent) if p else None
                if parent_op is not None and implies(parent_op, olddep_name):
                    return True
            return False

        ret = type(self)(volume=self)
        ret.dependent_names = [op.name for op in ops]
        for old in self.dependent_names:
            if not any(implies(n, old) for n in ops):
                ret.dependent_names.append(old)
        return ret
