# picotron/pipeline_parallel: only its p2p layer is on the hot path
