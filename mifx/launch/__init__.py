"""Training-job specs and a single-node multi-process launcher (one process per MI355X).

Replaces the reference's TFJob / PyTorchJob / MPIJob operators for single-node data/tensor
parallelism (`infrastructure/crd/tfjob-crd-v1.yaml:1-46`,
`notebooks/training-jobs/distributed-tensorflow-training-job.yaml`,
`pytorch-job.jsonnet:63-81`, `mpi-job.libsonnet:22-85`): the same manifests are accepted; every
replica becomes a local process with RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR=127.0.0.1 /
MASTER_PORT (torch.distributed over RCCL) and, for TFJob, a TF_CONFIG cluster spec. Every rank sees every GPU of
the node (LOCAL_RANK picks its own: the xGMI peer exchange and RCCL P2P need the peers visible); `restartPolicy`
OnFailure / Always / ExitCode relaunch the replica set from its checkpoint up to `backoffLimit` times, Never fails
fast (`tf-job-simple-v1beta2.jsonnet:45,71`)."""
from .job import JobSpec, ReplicaSpec, launch_local, to_indexed_job, validate  # noqa: F401
