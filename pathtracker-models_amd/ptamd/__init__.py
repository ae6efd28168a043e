"""ptamd — host side of the MI355X recurrent-cell library (bindings, autograd, data)."""
