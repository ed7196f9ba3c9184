"""Scalar dashboard (TensorBoard equivalent): mifx.board.server."""
