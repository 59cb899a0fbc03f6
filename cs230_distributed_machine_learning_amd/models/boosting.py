"""Placeholder: family registered later in the build."""
