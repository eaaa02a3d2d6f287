"""Agents over the GPU engine (reference: agents/)."""
