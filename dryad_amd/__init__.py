"""Dryad-AMD: an MI355X-native DAG data-parallel engine with the DryadLINQ programming model."""
__version__ = "0.1.0"
