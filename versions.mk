# Release versions (reference analogue: versions.mk:17-24).
MODULE := github.com/amd-mi355x/gpu-feature-discovery-amd
VERSION ?= v0.1.0
ROCM_VERSION := 7.2.0
UBUNTU_VERSION := 22.04
GIT_COMMIT ?= $(shell git describe --match="" --dirty --long --always 2>/dev/null || echo unknown)
IMAGE_NAME ?= registry.example.com/amd/gpu-feature-discovery-amd
